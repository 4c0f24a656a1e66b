#!/bin/bash
# Headline bench A/B in one GPU session: args are "ENV=VAL ..." arm specs separated by ';' ("" = default arm).
set -o pipefail
mkdir -p gpurun_out
B=${BATCH:-1024}
IFS=';' read -ra ARMS <<< "$1"
for arm in "${ARMS[@]}"; do
  echo "arm [$arm]"
  env $arm timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --batch $B 2> gpurun_out/bench_ab.err | tail -1 | cut -c1-160 || { tail -5 gpurun_out/bench_ab.err; exit 1; }
done
