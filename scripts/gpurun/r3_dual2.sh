#!/bin/bash
# GPU job (round 3): ResNet GPU tests after the dual-BN test fix, then the whole -m gpu suite.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_resnet_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/dual_tests.log 2>&1 || { grep -E "Error|assert" gpurun_out/dual_tests.log | cut -c1-3000 | tail -8; exit 1; }
tail -1 gpurun_out/dual_tests.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/fin_suite.log 2>&1 || { tail -60 gpurun_out/fin_suite.log; exit 1; }
tail -1 gpurun_out/fin_suite.log
