#!/bin/bash
# GPU job (round 3): LDS-DMA staged stem kernels -- tests, bench, profile.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_resnet_gpu.py tests/test_gemm_conv_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/stem2_tests.log 2>&1 || { tail -40 gpurun_out/stem2_tests.log; exit 1; }
tail -1 gpurun_out/stem2_tests.log
bash scripts/gpurun/env_ab.sh "" || exit 1
bash scripts/gpurun/r3_prof.sh
