#!/bin/bash
# GPU job (round 5, final tree): ResNet-50 per-GPU batch 3072 vs 4096, alternating, 3 pairs
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_b4096b; rm -rf $O; mkdir -p $O
i=0
for b in 3072 4096 3072 4096 3072 4096; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py --batch $b --steps 20 --warmup 5 > $O/b${i}_$b.json 2> $O/b${i}_$b.err || { tail -20 $O/b${i}_$b.err; exit 1; }
  echo "b$b: $(python3 -c "import json,sys; r=json.load(open(sys.argv[1])); print(r['value'], r['ms_per_step'])" $O/b${i}_$b.json)"
done
