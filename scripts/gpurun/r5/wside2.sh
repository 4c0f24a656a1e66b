#!/bin/bash
# GPU job (round 5): does the side stream run concurrently at all? bench arms (serial / side prio 0 / side prio -1)
# at batch 1024, then a kernel trace of 3 steps with the side stream to measure overlap.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_wside2; rm -rf $O; mkdir -p $O
for arm in "0 0" "1 0" "1 -1" "0 0" "1 0" "1 -1"; do
  set -- $arm
  K8S_AMD_WGRAD_STREAM=$1 K8S_AMD_WGRAD_PRIO=$2 timeout -k 10 300 python -u bench.py --batch 1024 --steps 20 --warmup 5 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  echo "side=$1 prio=$2: $(python -c "import json; d=json.load(open('$O/b.json')); print(d['value'], d['ms_per_step'])")"
done
K8S_AMD_WGRAD_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o trace -- python -u bench.py --batch 1024 --steps 3 --warmup 2 > $O/p.log 2>&1 || { tail -20 $O/p.log; exit 1; }
find $O/prof -name "*kernel_trace.csv" | head -3
