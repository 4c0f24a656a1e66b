#!/bin/bash
# GPU job (round 3): attention numerics incl. the split dK/dV edge cases, then split-count A/B (default rule, 2, 8).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1 || { tail -40 gpurun_out/attn_tests.log; exit 1; }
tail -1 gpurun_out/attn_tests.log
for sp in 0 2 8; do
  K8S_AMD_FA_DKV_SPLIT=$sp timeout -k 10 200 python -u scripts/bench_attention.py > gpurun_out/attn_bench_sp$sp.jsonl 2> gpurun_out/attn_bench_sp$sp.err || { tail -20 gpurun_out/attn_bench_sp$sp.err; exit 1; }
  echo "split=$sp"; grep -o '"case": "[a-z0-9_]*".*"bwd_ms": [0-9.]*' gpurun_out/attn_bench_sp$sp.jsonl | sed 's/"B".*"bwd_ms"/ bwd_ms/'
done
