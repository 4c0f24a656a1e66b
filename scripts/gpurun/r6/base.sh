#!/bin/bash
# GPU job (round 6 start): whole GPU suite, smoke, default bench (b3072) and b1024 bench, b3072 step profile.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r6_base}; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/suite.log 2>&1 || { tail -40 $O/suite.log; exit 1; }
tail -1 $O/suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
timeout -k 10 400 python -u bench.py --batch 1024 > $O/bench1024.json 2> $O/bench1024.err || { tail -20 $O/bench1024.err; exit 1; }
cut -c1-300 $O/bench1024.json
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o rn -- python3 bench.py --steps 6 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/profile_report.py $(ls $O/prof/*kernel_trace.csv | head -1) --step-marker sgd_kernel --top 75 --title "ResNet-50 b3072, round 6 start" > $O/rn.md && head -14 $O/rn.md
