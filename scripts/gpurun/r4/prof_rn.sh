#!/bin/bash
# GPU job (round 4, end): steady-state kernel trace of the ResNet-50 b1024 bench step.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4_rn_end; rm -rf $O; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o rn -- python3 bench.py --steps 8 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/profile_report.py $(ls $O/prof/*kernel_trace.csv | head -1) --step-marker sgd_kernel --top 60 --title "ResNet-50 b1024, round 4 end" > $O/rn.md && head -14 $O/rn.md
