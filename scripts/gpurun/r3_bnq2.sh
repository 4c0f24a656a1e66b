#!/bin/bash
# GPU job (round 3): BatchNorm / ResNet GPU tests after a knob cleanup, then the bn1 -> conv2 normalize-on-load A/B
# (K8S_AMD_BN_ONLOAD=all vs the 1x1 default) with the current kernels.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_resnet_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/bnq_tests.log 2>&1 || { tail -30 gpurun_out/bnq_tests.log; exit 1; }
tail -1 gpurun_out/bnq_tests.log
bash scripts/gpurun/env_ab.sh "K8S_AMD_BN_ONLOAD=1x1" "K8S_AMD_BN_ONLOAD=all"
