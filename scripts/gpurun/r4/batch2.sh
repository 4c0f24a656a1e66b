#!/bin/bash
# GPU job (round 4): staged 3x3 + bn1 on load + knob removal + ZeRO bf16 pull -- tests, bench A/B, ZeRO update cost.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_conv3x3_gpu.py tests/test_resnet_gpu.py tests/test_gemm256_gpu.py tests/test_wgrad_stream_gpu.py tests/test_gemm_conv_gpu.py tests/test_attention_gpu.py tests/test_dist_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r4_b2_tests.log 2>&1 || { tail -40 gpurun_out/r4_b2_tests.log; exit 1; }
tail -2 gpurun_out/r4_b2_tests.log
bash scripts/gpurun/env_ab.sh "" "K8S_AMD_BN_ONLOAD=1x1" || exit 1
timeout -k 10 300 python -u scripts/bench_zero_update.py > gpurun_out/r4_zero_update.json 2> gpurun_out/r4_zero_update.err || { tail -20 gpurun_out/r4_zero_update.err; exit 1; }
cat gpurun_out/r4_zero_update.json
