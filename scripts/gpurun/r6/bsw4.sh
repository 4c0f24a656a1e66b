#!/bin/bash
# GPU job (round 6): BN-backward sums in the 4-wave kernel's dgrad copy-out (stage-3/4 bn2) -- tests, same-box A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_bsw4; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_conv_gpu.py -k "bnstats" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_resnet_gpu.py > $O/tests2.log 2>&1 || { tail -40 $O/tests2.log; exit 1; }
tail -2 $O/tests2.log
bash scripts/gpurun/r6/envab.sh r6_bsw4_ab 2 3072 "on:X=1" "off:K8S_AMD_BN_BSTATS_W4=0" || exit 1
bash scripts/gpurun/r6/envab.sh r6_bsw4_ab1k 2 1024 "on:X=1" "off:K8S_AMD_BN_BSTATS_W4=0"
