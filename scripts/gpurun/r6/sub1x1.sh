#!/bin/bash
# GPU job (round 6): subsampled downsample 1x1 (ops.conv.SUB1X1) and K = 512 on the 4-wave GEMM -- tests, bench A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_sub1x1; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_conv_gpu.py tests/test_resnet_gpu.py tests/test_gemm256_gpu.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
bash scripts/gpurun/r6/envab.sh r6_sub1x1_ab 2 3072 "base:X=1" "nosub:K8S_AMD_SUB1X1=0" "mink512:K8S_AMD_GEMM256_MINK=512"
