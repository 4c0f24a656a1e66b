#!/bin/bash
# GPU job: per-layer ResNet-50 roofline at the bench batch (scripts/layer_roofline.py).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/layer_roofline.py --batch ${1:-1024} > gpurun_out/roofline.jsonl 2> gpurun_out/roofline.err || { tail -30 gpurun_out/roofline.err; exit 1; }
tail -1 gpurun_out/roofline.jsonl
