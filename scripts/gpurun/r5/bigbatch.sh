#!/bin/bash
# GPU job (round 5): large-batch indexing check (duplicated half batch) + short-K kernel tests.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_bigbatch; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_resnet_gpu.py tests/test_gemm_short_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
