#!/bin/bash
# GPU job (round 6): ResNet-50 b1024 step profile on the final tree.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_prof1024_final; rm -rf $O; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o rn -- python3 bench.py --batch 1024 --steps 8 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/profile_report.py $(ls $O/prof/*kernel_trace.csv | head -1) --step-marker sgd_kernel --top 90 --title "ResNet-50 b1024, round 6 (final tree)" > $O/rn.md && head -16 $O/rn.md
rm -rf $O/prof
