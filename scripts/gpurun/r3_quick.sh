#!/bin/bash
# GPU job (round 3): new transport kernels, multi-rank paths on the GPU kernels, graph test, then the bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py::test_slice_sum_and_cast_bf16 tests/test_dist_gpu.py tests/test_graph_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r3_quick.log 2>&1 || { tail -60 gpurun_out/r3_quick.log; exit 1; }
tail -3 gpurun_out/r3_quick.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r3_bench.json 2> gpurun_out/r3_bench.err || { tail -30 gpurun_out/r3_bench.err; exit 1; }
cut -c1-400 gpurun_out/r3_bench.json
