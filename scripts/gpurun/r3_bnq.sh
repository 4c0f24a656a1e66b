#!/bin/bash
# GPU job (round 3): BatchNorm / ResNet GPU tests after a knob cleanup.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_resnet_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/bnq_tests.log 2>&1 || { tail -30 gpurun_out/bnq_tests.log; exit 1; }
tail -1 gpurun_out/bnq_tests.log
