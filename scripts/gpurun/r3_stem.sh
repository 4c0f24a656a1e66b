#!/bin/bash
# GPU job (round 3): stem kernels (LDS-tiled s2d conv + weight gradient, fused BN + ReLU + max pool) -- tests, A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_resnet_gpu.py tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/stem_tests.log 2>&1 || { tail -40 gpurun_out/stem_tests.log; exit 1; }
tail -1 gpurun_out/stem_tests.log
bash scripts/gpurun/env_ab.sh "K8S_AMD_STEM_CONV=0" "K8S_AMD_STEM_CONV=1" || exit 1
bash scripts/gpurun/r3_prof.sh
