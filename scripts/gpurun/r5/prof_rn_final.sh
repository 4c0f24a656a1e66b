#!/bin/bash
# GPU job (round 5): ResNet-50 b3072 step profile on the final tree (bench code path)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_prof_rn_final; rm -rf $O; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/p -o rn -- python3 bench.py --steps 4 --warmup 2 > $O/p.log 2>&1 || { tail -20 $O/p.log; exit 1; }
python3 scripts/profile_report.py $(ls $O/p/*kernel_trace.csv | head -1) --step-marker sgd_kernel --top 75 --title "ResNet-50 b3072 (bench default), round-5 final tree" > $O/rn.md && head -16 $O/rn.md
rm -rf $O/p
