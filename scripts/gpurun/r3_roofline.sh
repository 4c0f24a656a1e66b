#!/bin/bash
# GPU job (round 3): per-layer ResNet-50 roofline at b1024.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/layer_roofline.py --batch 1024 > gpurun_out/roofline.jsonl 2> gpurun_out/roofline.err || { tail -30 gpurun_out/roofline.err; exit 1; }
tail -1 gpurun_out/roofline.jsonl
