#!/bin/bash
# GPU job (round 4): short-K streaming GEMM -- its tests, the conv / GEMM suites it now serves, and the ResNet-50
# 1x1 shapes with it on / off (K8S_AMD_GEMM_SHORT).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_short_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_gsk_tests.log 2>&1 || { tail -40 gpurun_out/r4_gsk_tests.log; exit 1; }
tail -1 gpurun_out/r4_gsk_tests.log
timeout -k 10 300 python -u -m pytest tests/test_gemm_conv_gpu.py tests/test_resnet_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_gsk_tests2.log 2>&1 || { tail -40 gpurun_out/r4_gsk_tests2.log; exit 1; }
tail -1 gpurun_out/r4_gsk_tests2.log
timeout -k 10 300 python -u scripts/gpurun/r4/c1x1.py > gpurun_out/r4_gsk_on.jsonl 2> gpurun_out/r4_gsk.err || { tail -30 gpurun_out/r4_gsk.err; exit 1; }
K8S_AMD_GEMM_SHORT=0 timeout -k 10 300 python -u scripts/gpurun/r4/c1x1.py > gpurun_out/r4_gsk_off.jsonl 2>> gpurun_out/r4_gsk.err || { tail -30 gpurun_out/r4_gsk.err; exit 1; }
cat gpurun_out/r4_gsk_on.jsonl gpurun_out/r4_gsk_off.jsonl
