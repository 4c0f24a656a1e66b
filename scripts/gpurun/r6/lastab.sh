#!/bin/bash
# GPU job (round 6): the kept BN-sums forms (stem pool, stage-4 tile kernel) on vs off at b3072 and b1024, then the
# b3072 step profile of the default tree.
set -o pipefail
export TMPDIR=/tmp
bash scripts/gpurun/r6/envab.sh r6_lastab3072 2 3072 "on:X=1" "off:K8S_AMD_BN_BSTATS_POOL=0 K8S_AMD_BN_BSTATS_TILE_MASK=0" || exit 1
bash scripts/gpurun/r6/envab.sh r6_lastab1024 2 1024 "on:X=1" "off:K8S_AMD_BN_BSTATS_POOL=0 K8S_AMD_BN_BSTATS_TILE_MASK=0" || exit 1
O=gpurun_out/r6_lastprof; rm -rf $O; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o rn -- python3 bench.py --steps 6 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/profile_report.py $(ls $O/prof/*kernel_trace.csv | head -1) --step-marker sgd_kernel --top 90 --title "ResNet-50 b3072, round 6 (final tree)" > $O/rn.md && head -16 $O/rn.md
rm -rf $O/prof
