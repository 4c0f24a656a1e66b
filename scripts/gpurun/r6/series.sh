#!/bin/bash
# GPU job (round 6): the bench series on the current tree (b3072 default and b1024, two runs each, alternating) and
# stock PyTorch-ROCm ResNet-50 at b3072 in MIOpen immediate mode (no Find search: the FAST find at b3072 did not
# finish within 1100 s, gpurun_out/r6_stock), for a same-batch ratio.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r6_series}; rm -rf $O; mkdir -p $O
for r in 1 2; do
  for b in 3072 1024; do
    timeout -k 10 300 python -u bench.py --batch $b --steps 20 --warmup 5 > $O/b${b}_$r.json 2> $O/b${b}_$r.err || { tail -20 $O/b${b}_$r.err; exit 1; }
    echo "b$b rep $r: $(python3 -c "import json,sys; r=json.load(open(sys.argv[1])); print(r['value'], r['ms_per_step'])" $O/b${b}_$r.json)"
  done
done
( while sleep 50; do date +%s >> $O/heartbeat.txt; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 700 python -u benchmarks/stock_baselines.py --model resnet50 --batch 3072 --steps 10 --warmup 3 --no-find > $O/stock_b3072_immediate.json 2> $O/stock_b3072_immediate.err || { tail -5 $O/stock_b3072_immediate.err; exit 1; }
cat $O/stock_b3072_immediate.json
