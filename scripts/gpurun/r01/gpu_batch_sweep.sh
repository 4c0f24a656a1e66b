#!/bin/bash
# Per-GPU batch sweep of the ResNet-50 bench (b768, b1024), autotune choices kept for the seed table.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sweep
export TMPDIR=/tmp
for b in 768 1024; do
  K8S_AMD_AUTOTUNE_VERBOSE=1 timeout -k 10 600 python bench.py --steps 20 --warmup 5 --batch $b > gpurun_out/sweep/bench$b.log 2> gpurun_out/sweep/bench$b.err || { tail -20 gpurun_out/sweep/bench$b.err; exit 1; }
  cat gpurun_out/sweep/bench$b.log
done
