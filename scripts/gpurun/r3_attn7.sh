#!/bin/bash
# GPU job (round 3): 8-wave forward A/B: K8S_AMD_FA_FWD8 = 0 (4 waves, 2 stages), 1 (8 waves, 3 stages), 2 (8 waves,
# 2 stages); numerics under each.
set -o pipefail
mkdir -p gpurun_out
for f in 1 2; do
  K8S_AMD_FA_FWD8=$f timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_tests_f$f.log 2>&1 || { tail -40 gpurun_out/attn_tests_f$f.log; exit 1; }
  tail -1 gpurun_out/attn_tests_f$f.log
done
for f in 0 1 2 0 1 2; do
  K8S_AMD_FA_FWD8=$f timeout -k 10 200 python -u scripts/bench_attention.py > gpurun_out/attn_bench_f$f.jsonl 2> gpurun_out/attn_bench_f$f.err || { tail -20 gpurun_out/attn_bench_f$f.err; exit 1; }
  echo "fwd8=$f"; grep -o '"case": "[a-z0-9_]*".*"fwd_ms": [0-9.]*' gpurun_out/attn_bench_f$f.jsonl | sed 's/"B".*"fwd_ms"/ fwd_ms/' | grep -v bert
done
