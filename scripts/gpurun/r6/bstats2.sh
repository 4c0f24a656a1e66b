#!/bin/bash
# GPU job (round 6): BatchNorm-backward sums in the dgrad epilogues (identity-block 1x1 with the masked addend,
# stride-1 3x3 for bn1) -- kernel + ResNet tests, same-box bench A/B (K8S_AMD_BN_BSTATS), then the b3072 step profile.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r6_bstats2}; rm -rf $O; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gemm_conv_gpu.py tests/test_resnet_gpu.py > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
bash scripts/gpurun/r6/envab.sh ${1:-r6_bstats2}_ab 2 3072 "on:K8S_AMD_BN_BSTATS=1" "off:K8S_AMD_BN_BSTATS=0" || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o rn -- python3 bench.py --steps 6 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/profile_report.py $(ls $O/prof/*kernel_trace.csv | head -1) --step-marker sgd_kernel --top 75 --title "ResNet-50 b3072, round 6, BN-backward sums in the dgrad epilogues" > $O/rn.md && head -45 $O/rn.md
rm -rf $O/prof
