#!/bin/bash
# GPU job (round 6): which BatchNorm-backward-sums epilogues pay, same box, arms alternating.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_bstats3; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_conv_gpu.py -k "bnstats" tests/test_resnet_gpu.py -k "bn_backward_sums" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash scripts/gpurun/r6/envab.sh r6_bstats3_ab 2 3072 "all:X=1" "no3x3:K8S_AMD_BN_BSTATS_3X3=0" "nogemm:K8S_AMD_BN_BSTATS_GEMM=0" "short:K8S_AMD_BN_BSTATS_3X3=0 K8S_AMD_BN_BSTATS_GEMM=0" "off:K8S_AMD_BN_BSTATS=0"
