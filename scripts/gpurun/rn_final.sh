#!/bin/bash
# GPU job: headline bench twice, then the steady-state kernel trace of it.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_rn50
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/rn_bench.json 2> gpurun_out/rn_bench.err || { tail -20 gpurun_out/rn_bench.err; exit 1; }
  cut -c1-200 gpurun_out/rn_bench.json
done
bash scripts/gpurun/prof_resnet_steady.sh
