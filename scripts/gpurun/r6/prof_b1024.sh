#!/bin/bash
# GPU job (round 6): step profiles at b1024 and b3072 on the current tree (per-kernel, for the batch comparison).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r6_prof_b1024}; rm -rf $O; mkdir -p $O
for b in 1024 3072; do
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof$b -o rn -- python3 bench.py --batch $b --steps 6 --warmup 3 > $O/prof$b.log 2>&1 || { tail -20 $O/prof$b.log; exit 1; }
  python3 scripts/profile_report.py $(ls $O/prof$b/*kernel_trace.csv | head -1) --step-marker sgd_kernel --top 90 --title "ResNet-50 b$b, round 6" > $O/rn$b.md && head -16 $O/rn$b.md
  rm -rf $O/prof$b
done
