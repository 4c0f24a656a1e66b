#!/bin/bash
# GPU job (round 4): op placement variants of the 4-wave NT GEMM, same box, alternating processes.
set -o pipefail
mkdir -p gpurun_out
K8S_AMD_W4_SPREAD=2 timeout -k 10 300 python -u -m pytest tests/test_gemm256_gpu.py -x -q --timeout 120 --timeout-method thread -k "w4" > gpurun_out/r4_w4sp2_tests.log 2>&1 || { tail -30 gpurun_out/r4_w4sp2_tests.log; exit 1; }
tail -1 gpurun_out/r4_w4sp2_tests.log
for i in 1 2; do
  for sp in 1 2; do
    K8S_AMD_W4_SPREAD=$sp timeout -k 10 120 python -u scripts/gpurun/r4/gemm_time.py >> gpurun_out/r4_w4sp2.jsonl 2>> gpurun_out/r4_w4sp2.err || { tail -20 gpurun_out/r4_w4sp2.err; exit 1; }
  done
done
cat gpurun_out/r4_w4sp2.jsonl
