#!/bin/bash
# GPU job (round 5): the side-stream weight-gradient test with the short-K GEMM's stores deferred / not deferred
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_gskdefer2; rm -rf $O; mkdir -p $O
for v in 0 1 1; do
  K8S_AMD_GSK_DEFER=$v timeout -k 10 200 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_resnet_gpu.py -k "side_stream or gradients" > $O/t_$v.log 2>&1; echo "defer=$v rc=$? $(tail -1 $O/t_$v.log)"
done
K8S_AMD_GSK_DEFER=1 timeout -k 10 200 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gemm_short_gpu.py > $O/gs.log 2>&1; echo "gemm_short defer=1 rc=$? $(tail -1 $O/gs.log)"
