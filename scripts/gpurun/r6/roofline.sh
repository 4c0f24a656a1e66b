#!/bin/bash
# GPU job (round 6): per-layer roofline at b3072 with fused-aware floors (scripts/layer_roofline.py).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r6_roofline}; rm -rf $O; mkdir -p $O
( while sleep 50; do date +%s >> $O/heartbeat.txt; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u scripts/layer_roofline.py --batch 3072 --reps 5 > $O/roofline.jsonl 2> $O/roofline.err || { tail -20 $O/roofline.err; exit 1; }
tail -1 $O/roofline.jsonl
