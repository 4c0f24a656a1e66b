#!/bin/bash
# GPU job: the multi-rank path on the GPU kernels (2 ranks sharing the box's one GPU over gloo).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_dist_gpu.py > gpurun_out/dist_test.log 2>&1 || { tail -60 gpurun_out/dist_test.log; exit 1; }
tail -4 gpurun_out/dist_test.log
