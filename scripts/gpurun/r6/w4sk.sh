#!/bin/bash
# GPU job (round 6): deep-K 1x1 statistics forwards with a partial last wave on the 4-wave kernel's stream-K tail
# (K8S_AMD_W4_STATS_SK) -- tests, then same-box A/B at b1024 and b3072.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_w4sk; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_conv_gpu.py -k "w4_stats or bnstats or conv_fwd" tests/test_resnet_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash scripts/gpurun/r6/envab.sh r6_w4sk_ab1k 3 1024 "on:X=1" "off:K8S_AMD_W4_STATS_SK=0" || exit 1
bash scripts/gpurun/r6/envab.sh r6_w4sk_ab 2 3072 "on:X=1" "off:K8S_AMD_W4_STATS_SK=0"
