#!/bin/bash
# GPU job (round 6): the stem BN + two-BN sums in the tile-kernel masked dgrad -- tests, A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_bsstr; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_gemm_conv_gpu.py -k "bnstats or strided" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_resnet_gpu.py > $O/tests2.log 2>&1 || { tail -40 $O/tests2.log; exit 1; }
tail -2 $O/tests2.log
bash scripts/gpurun/r6/envab.sh r6_bsstr_ab 2 3072 "on:X=1" "nostr:K8S_AMD_BN_BSTATS_STRIDED=0" "noshort:K8S_AMD_BN_BSTATS_TILE_SHORT=0" "off:K8S_AMD_BN_BSTATS_TILE_MASK=0 K8S_AMD_BN_BSTATS_STRIDED=0"
