#!/bin/bash
# GPU job (round 3): attention A/B (new 32x32 forward), stream-order A/B on the headline bench, stock ResNet-50 with
# MIOpen FAST find (heartbeat file so the silent find is not taken for a hang).
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpurun/r3_attn.sh || exit 1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_conv_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/it2_tests.log 2>&1 || { tail -40 gpurun_out/it2_tests.log; exit 1; }
tail -1 gpurun_out/it2_tests.log
bash scripts/gpurun/env_ab.sh "K8S_AMD_STREAM_ORDER=1" "K8S_AMD_STREAM_ORDER=2" || exit 1
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) &
HB=$!
timeout -k 10 600 python -u benchmarks/stock_baselines.py --model resnet50 --batch 1024 --steps 10 --warmup 3 --miopen-find-mode FAST > gpurun_out/stock/resnet50_fast.json 2> gpurun_out/stock/resnet50_fast.err
echo "stock resnet rc=$? $(grep '^{' gpurun_out/stock/resnet50_fast.json | cut -c1-250)"
kill $HB
