#!/bin/bash
# rocprofv3 kernel-trace summary of the headline bench (ResNet-50, batch 1024/GPU) + the bench line itself.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B=${1:-1024}
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --batch $B > gpurun_out/bench_b$B.json 2> gpurun_out/bench_b$B.err && cat gpurun_out/bench_b$B.json &&
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rn$B -o rn -- python3 bench.py --steps 4 --warmup 2 --batch $B > gpurun_out/prof_rn$B.log 2>&1
echo "prof rc=$?"
