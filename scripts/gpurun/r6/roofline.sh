#!/bin/bash
# GPU job (round 6): per-layer roofline at b3072 with fused-aware floors (scripts/layer_roofline.py).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_roofline; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u scripts/layer_roofline.py --batch 3072 --reps 5 > $O/roofline.jsonl 2> $O/roofline.err || { tail -20 $O/roofline.err; exit 1; }
tail -1 $O/roofline.jsonl
