#!/bin/bash
# GPU job (round 5): per-GPU batch sweep of the headline bench (weak scaling; 288 GB HBM per GPU).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_batch; rm -rf $O; mkdir -p $O
for b in ${BATCHES:-1024 2048 3072}; do
  timeout -k 10 400 python -u bench.py --batch $b --steps 12 --warmup 4 > $O/b$b.json 2> $O/b$b.err || { tail -20 $O/b$b.err; exit 1; }
  cut -c1-160 $O/b$b.json
  grep -o '"peak_mem_gb": [0-9.]*' $O/b$b.json
done
