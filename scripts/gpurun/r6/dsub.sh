#!/bin/bash
# GPU job (round 6): 1x1 / stride-2 data gradients as a compact GEMM + upsample-add (K8S_AMD_DGRAD_SUB1X1) -- tests,
# then a same-box bench A/B at b3072 and b1024.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_dsub; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_conv_gpu.py -k "strided or bnstats" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_resnet_gpu.py > $O/tests2.log 2>&1 || { tail -40 $O/tests2.log; exit 1; }
tail -2 $O/tests2.log
bash scripts/gpurun/r6/envab.sh r6_dsub_ab 2 3072 "on:X=1" "off:K8S_AMD_DGRAD_SUB1X1=0" || exit 1
bash scripts/gpurun/r6/envab.sh r6_dsub_ab1k 2 1024 "on:X=1" "off:K8S_AMD_DGRAD_SUB1X1=0"
