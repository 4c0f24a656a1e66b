#!/bin/bash
# GPU job (round 6): the downsample input's subsample written by the previous BN apply (K8S_AMD_SUB2_FUSED).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_sub2; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_resnet_gpu.py tests/test_kernels_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash scripts/gpurun/r6/envab.sh r6_sub2_ab 3 3072 "on:X=1" "off:K8S_AMD_SUB2_FUSED=0"
