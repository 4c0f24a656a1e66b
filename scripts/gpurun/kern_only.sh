#!/bin/bash
# GPU job: kernel tests only.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py > gpurun_out/kern_test.log 2>&1 || { tail -40 gpurun_out/kern_test.log; exit 1; }
tail -1 gpurun_out/kern_test.log
