#!/bin/bash
# GPU job (round 4): bn1 normalised on load by the staged 3x3 kernels + knob removal -- kernel / model tests, bench A/B.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_conv3x3_gpu.py tests/test_resnet_gpu.py tests/test_gemm256_gpu.py tests/test_wgrad_stream_gpu.py tests/test_gemm_conv_gpu.py tests/test_attention_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4_onload_tests.log 2>&1 || { tail -40 gpurun_out/r4_onload_tests.log; exit 1; }
tail -2 gpurun_out/r4_onload_tests.log
bash scripts/gpurun/env_ab.sh "" "K8S_AMD_BN_ONLOAD=1x1" || exit 1
