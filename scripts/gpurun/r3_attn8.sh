#!/bin/bash
# GPU job (round 3): forward scheduling variants (K8S_AMD_FA_FWD_VAR: 0 = rescale branch, 1 = unconditional rescale,
# one basic block per tile), numerics for variant 1, alternating benchmark runs.
set -o pipefail
mkdir -p gpurun_out
K8S_AMD_FA_FWD_VAR=1 timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_tests_v1.log 2>&1 || { tail -40 gpurun_out/attn_tests_v1.log; exit 1; }
tail -1 gpurun_out/attn_tests_v1.log
for v in 0 1 0 1; do
  K8S_AMD_FA_FWD_VAR=$v timeout -k 10 200 python -u scripts/bench_attention.py > gpurun_out/attn_bench_v$v.jsonl 2> gpurun_out/attn_bench_v$v.err || { tail -20 gpurun_out/attn_bench_v$v.err; exit 1; }
  echo "var=$v"; grep -o '"case": "[a-z0-9_]*".*"fwd_ms": [0-9.]*' gpurun_out/attn_bench_v$v.jsonl | sed 's/"B".*"fwd_ms"/ fwd_ms/' | grep -v "bert\|d64"
done
