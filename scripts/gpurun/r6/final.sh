#!/bin/bash
# GPU job (round 6): whole GPU suite, smoke, bench at b3072 / b1024, then the b3072 step profile.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r6_final}
bash scripts/gpurun/r6/suite.sh ${1:-r6_final} || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o rn -- python3 bench.py --steps 6 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/profile_report.py $(ls $O/prof/*kernel_trace.csv | head -1) --step-marker sgd_kernel --top 90 --title "ResNet-50 b3072, round 6 (final tree)" > $O/rn.md && head -24 $O/rn.md
rm -rf $O/prof
