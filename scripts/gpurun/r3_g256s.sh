#!/bin/bash
# GPU job (round 3): split-K on the 256 x 256 GEMM -- tests, A/B on the headline bench, profile.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_conv_gpu.py tests/test_resnet_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/g256s_tests.log 2>&1 || { tail -40 gpurun_out/g256s_tests.log; exit 1; }
tail -1 gpurun_out/g256s_tests.log
bash scripts/gpurun/env_ab.sh "K8S_AMD_G256_SPLITK=0" "" || exit 1
bash scripts/gpurun/r3_prof.sh
