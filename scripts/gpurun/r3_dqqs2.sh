#!/bin/bash
# GPU job (round 3): dQ with 32 queries per wave at D = 128 (K8S_AMD_FA_DQ_QS2=1) vs default, after the swizzle fix.
set -o pipefail
mkdir -p gpurun_out
for v in 0 1 0 1; do
  K8S_AMD_FA_DQ_QS2=$v timeout -k 10 200 python -u scripts/bench_attention.py > gpurun_out/attn_bench_q$v.jsonl 2> gpurun_out/attn_bench_q$v.err || { tail -20 gpurun_out/attn_bench_q$v.err; exit 1; }
  echo "qs2=$v"; grep -o '"case": "[a-z0-9_]*".*"bwd_ms": [0-9.]*' gpurun_out/attn_bench_q$v.jsonl | sed 's/"B".*"bwd_ms"/ bwd_ms/' | grep -v "bert\|d64"
done
