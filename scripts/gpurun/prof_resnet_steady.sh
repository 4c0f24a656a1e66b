#!/bin/bash
# GPU job: rocprofv3 kernel trace of the headline bench (ResNet-50 b1024); steady-state report between SGD launches.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rn50 -o rn50 -- python3 bench.py --steps 6 --warmup 2 > gpurun_out/prof_rn50.log 2>&1
echo "prof rc=$?"
grep '^{' gpurun_out/prof_rn50.log | cut -c1-160
