#!/bin/bash
# GPU job (round 6): deep 1x1 forwards on the 4-wave GEMM with the BN-statistics epilogue -- tests, bench A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_w4stats; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_conv_gpu.py tests/test_resnet_gpu.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
bash scripts/gpurun/r6/envab.sh r6_w4stats_ab 2 3072 "w4s:K8S_AMD_W4_STATS=1" "off:K8S_AMD_W4_STATS=0" "w4s1024:K8S_AMD_W4_STATS_MINK=1024"
