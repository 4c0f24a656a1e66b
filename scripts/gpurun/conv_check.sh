#!/bin/bash
# GPU job: GEMM / conv / ResNet tests, then the headline bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_conv_gpu.py tests/test_gemm256_gpu.py tests/test_resnet_gpu.py tests/test_wgrad_stream_gpu.py > gpurun_out/cc_test.log 2>&1 || { tail -40 gpurun_out/cc_test.log; exit 1; }
tail -1 gpurun_out/cc_test.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
cut -c1-200 gpurun_out/bench.json
