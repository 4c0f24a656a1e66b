#!/bin/bash
# GPU job (round 6): stage-4 (7 x 7) 3x3 weight gradients on the tiled kernel (K8S_AMD_WG3_7X7) -- tests, A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_wg7; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_conv_gpu.py -k "wgrad" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_resnet_gpu.py -k "gradients or large_batch" > $O/tests2.log 2>&1 || { tail -40 $O/tests2.log; exit 1; }
tail -2 $O/tests2.log
bash scripts/gpurun/r6/envab.sh r6_wg7_ab 3 3072 "on:X=1" "off:K8S_AMD_WG3_7X7=0"
