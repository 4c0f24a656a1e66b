#!/bin/bash
# GPU job (round 3): stock ResNet-50 b1024 with MIOpen FAST find + cudnn.benchmark (a heartbeat file keeps the
# silent search from being taken for a hang).
set -o pipefail
mkdir -p gpurun_out/stock
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 1100 python -u benchmarks/stock_baselines.py --model resnet50 --batch 1024 --steps 10 --warmup 3 --miopen-find-mode FAST > gpurun_out/stock/resnet50_fast.json 2> gpurun_out/stock/resnet50_fast.err
echo "stock resnet rc=$? $(grep '^{' gpurun_out/stock/resnet50_fast.json | cut -c1-250)"
