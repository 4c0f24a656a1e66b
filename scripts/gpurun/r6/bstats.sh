#!/bin/bash
# GPU job (round 6): BatchNorm-backward sums in the identity-block dgrad epilogue (gemm_short.hip EPI 3 / 4,
# ops.nn.BnStatLink) -- kernel + model tests, then a same-box bench A/B (K8S_AMD_BN_BSTATS) and a stock ResNet-50
# b3072 run in MIOpen immediate mode (the FAST find at b3072 did not finish within 1100 s).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_bstats; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gemm_conv_gpu.py -k "bnstats or from_sums or masked_addend" tests/test_resnet_gpu.py > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
bash scripts/gpurun/r6/envab.sh r6_bstats_ab 2 3072 "on:K8S_AMD_BN_BSTATS=1" "off:K8S_AMD_BN_BSTATS=0"
