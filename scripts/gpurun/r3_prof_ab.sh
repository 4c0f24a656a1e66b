#!/bin/bash
# GPU job (round 3): rocprofv3 kernel stats of the bench with the bn2 apply normalised on load (1x1) vs not (0).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for mode in 0 1x1; do
  K8S_AMD_BN_ONLOAD=$mode timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ab_$mode -o rn -- python3 bench.py --steps 6 --warmup 2 > gpurun_out/prof_ab_$mode.log 2>&1 || { tail -20 gpurun_out/prof_ab_$mode.log; exit 1; }
  grep '^{' gpurun_out/prof_ab_$mode.log | cut -c1-120
done
