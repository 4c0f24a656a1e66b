#!/bin/bash
# GPU job: ResNet A/B against abtest/old, then a steady-state kernel trace of the bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpurun/tree_ab.sh &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rn50 -o rn50 -- python3 bench.py --steps 6 --warmup 2 > gpurun_out/prof_rn50.log 2>&1
echo "prof rc=$?"
