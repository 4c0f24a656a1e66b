#!/bin/bash
# Strided dgrad with the residual add fused: GEMM/conv + ResNet GPU tests, bench (+ autotune choices), profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/dacc
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gemm_conv_gpu.py tests/test_resnet_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/dacc/pytest.log 2>&1 || { tail -30 gpurun_out/dacc/pytest.log; exit 1; }
tail -2 gpurun_out/dacc/pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/dacc/bench.log 2> gpurun_out/dacc/bench.err || { tail -20 gpurun_out/dacc/bench.err; exit 1; }
cat gpurun_out/dacc/bench.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --batch 256 > gpurun_out/dacc/bench256.log 2> gpurun_out/dacc/bench256.err && cat gpurun_out/dacc/bench256.log &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dacc/prof -o run -- python bench.py --steps 5 --warmup 3 > gpurun_out/dacc/prof.log 2>&1 && echo prof ok
