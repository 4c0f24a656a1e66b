#!/bin/bash
# GPU job (round 4): kernel-stats profiles of the bench with bn1 on load (default) and applied (K8S_AMD_BN_ONLOAD=1x1).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r4_prof_a gpurun_out/r4_prof_b
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4_prof_a -o a -- python3 bench.py --steps 6 --warmup 2 > gpurun_out/r4_prof_a.log 2>&1 || { tail -5 gpurun_out/r4_prof_a.log; exit 1; }
export K8S_AMD_BN_ONLOAD=1x1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4_prof_b -o b -- python3 bench.py --steps 6 --warmup 2 > gpurun_out/r4_prof_b.log 2>&1 || { tail -5 gpurun_out/r4_prof_b.log; exit 1; }
python3 scripts/kstats_diff.py $(find gpurun_out/r4_prof_a -name "*kernel_stats.csv") $(find gpurun_out/r4_prof_b -name "*kernel_stats.csv") --steps 8 --top 25
