#!/bin/bash
# GPU job (round 6): the 1x1 tile-kernel BN-sums dgrad at 3 blocks / CU (x partly prefetched) -- test, same-box A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_bsgemm; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_conv_gpu.py -k "bnstats" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash scripts/gpurun/r6/envab.sh r6_bsgemm_ab 3 3072 "on:X=1" "nogemm:K8S_AMD_BN_BSTATS_GEMM=0"
