#!/bin/bash
# rocprofv3 kernel-trace summaries of the headline bench under two environments (A/B of a kernel path):
#   bash scripts/gpurun/prof_ab.sh "ENV=A" "ENV=B"
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for arm in "$1" "$2"; do
  i=$((i+1))
  echo "arm $i [$arm]"
  env $arm timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ab$i -o ab -- python3 bench.py --steps 4 --warmup 2 > gpurun_out/prof_ab$i.log 2>&1 || { tail -20 gpurun_out/prof_ab$i.log; exit 1; }
  grep metric gpurun_out/prof_ab$i.log | cut -c1-150
done
