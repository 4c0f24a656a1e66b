#!/bin/bash
# GPU job (round 4): persistent 4-wave GEMM A/B (K8S_AMD_W4_PERSIST=1 vs 0), same box, plus the gemm256 tests.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm256_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_w4p_tests.log 2>&1 || { tail -30 gpurun_out/r4_w4p_tests.log; exit 1; }
tail -1 gpurun_out/r4_w4p_tests.log
S="4096,28672,4096 4096,4096,14336 4096,6144,4096 4096,4096,4096 8192,8192,8192 4096,14336,4096 8192,768,3072 8192,3072,768"
for r in 1 2; do
  for p in 0 1; do
    K8S_AMD_W4_PERSIST=$p timeout -k 10 200 python -u scripts/gpurun/r4/gemm_time.py $S >> gpurun_out/r4_w4p.jsonl 2>> gpurun_out/r4_w4p.err || { tail -30 gpurun_out/r4_w4p.err; exit 1; }
  done
done
cat gpurun_out/r4_w4p.jsonl
