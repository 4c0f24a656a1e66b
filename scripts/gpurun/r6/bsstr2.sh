#!/bin/bash
# GPU job (round 6): sub-grid BN-sums epilogue with x / bits loaded up front -- tests, then the strided relu-kind
# sums (K8S_AMD_BN_BSTATS_STRIDED=1) against the default.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_bsstr2; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_conv_gpu.py -k "bnstats or strided or stage_entry" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
K8S_AMD_BN_BSTATS_STRIDED=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_resnet_gpu.py > $O/tests2.log 2>&1 || { tail -40 $O/tests2.log; exit 1; }
tail -2 $O/tests2.log
bash scripts/gpurun/r6/envab.sh r6_bsstr2_ab 3 3072 "def:X=1" "str:K8S_AMD_BN_BSTATS_STRIDED=1"
