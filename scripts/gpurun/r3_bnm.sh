#!/bin/bash
# GPU job (round 3): residual-BN backward order A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k bn > gpurun_out/bnm_tests.log 2>&1 || { tail -40 gpurun_out/bnm_tests.log; exit 1; }
K8S_AMD_BN_MASKED_PLAIN=2 timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k bn >> gpurun_out/bnm_tests.log 2>&1 || { tail -40 gpurun_out/bnm_tests.log; exit 1; }
tail -1 gpurun_out/bnm_tests.log
bash scripts/gpurun/env_ab.sh "" "K8S_AMD_BN_MASKED_PLAIN=2" || exit 1
