#!/bin/bash
# GPU job (round 6): ResNet GPU tests, then the ResNet-50 b3072 step profile on the current tree.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r6_prof_rn2}; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_resnet_gpu.py > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o rn -- python3 bench.py --steps 6 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/profile_report.py $(ls $O/prof/*kernel_trace.csv | head -1) --step-marker sgd_kernel --top 75 --title "ResNet-50 b3072, round 6 ${1:-}" > $O/rn.md && head -60 $O/rn.md
rm -rf $O/prof
