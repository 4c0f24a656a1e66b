#!/bin/bash
# GPU job (round 3): steady-state rocprofv3 kernel trace of the headline bench (ResNet-50 b1024).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof3
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof3 -o rn -- python3 bench.py --steps 6 --warmup 2 > gpurun_out/prof3.log 2>&1 || { tail -20 gpurun_out/prof3.log; exit 1; }
grep '^{' gpurun_out/prof3.log | cut -c1-160
