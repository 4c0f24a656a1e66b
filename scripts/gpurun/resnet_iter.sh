#!/bin/bash
# GPU job: ResNet GPU tests, then bench A/B against abtest/old (new, old, new, old).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_resnet_gpu.py tests/test_gemm_conv_gpu.py > gpurun_out/rn_test.log 2>&1 || { tail -40 gpurun_out/rn_test.log; exit 1; }
tail -1 gpurun_out/rn_test.log
bash scripts/gpurun/tree_ab.sh
