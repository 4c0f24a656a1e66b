#!/bin/bash
# GPU job (round 4): find the ResNet-50 bench regression -- env A/B of the new paths, then a kernel-stats profile.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpurun/env_ab.sh "" "K8S_AMD_CONV3X3=0" "K8S_AMD_GEMM256_SK=0" || exit 1
rm -rf gpurun_out/r4_rn_prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4_rn_prof -o rn -- python3 bench.py --steps 6 --warmup 2 > gpurun_out/r4_rn_prof.log 2>&1 || { tail -20 gpurun_out/r4_rn_prof.log; exit 1; }
f=$(find gpurun_out/r4_rn_prof -name "*kernel_stats.csv" | head -1); head -25 "$f" | cut -d, -f1-4 | cut -c1-200
