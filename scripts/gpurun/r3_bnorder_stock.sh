#!/bin/bash
# GPU job (round 3): BN kernel tests, BN pass-order A/B on the headline bench, then the stock PyTorch-ROCm baselines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_conv_gpu.py -x -q --timeout 120 --timeout-method thread -k "bn or resnet" > gpurun_out/bno_tests.log 2>&1 || { tail -40 gpurun_out/bno_tests.log; exit 1; }
tail -1 gpurun_out/bno_tests.log
K8S_AMD_BN_ORDER=0 timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "bn" > gpurun_out/bno_tests0.log 2>&1 || { tail -40 gpurun_out/bno_tests0.log; exit 1; }
tail -1 gpurun_out/bno_tests0.log
bash scripts/gpurun/env_ab.sh "K8S_AMD_BN_ORDER=0" "K8S_AMD_BN_ORDER=7" "K8S_AMD_BN_ORDER=1" || exit 1
bash scripts/gpurun/r3_stock.sh
