#!/bin/bash
# GPU job: stock PyTorch-ROCm ResNet-50 at the bench batch (1024) in MIOpen immediate mode (no Find), cold box.
set -o pipefail
mkdir -p gpurun_out
( while sleep 50; do date +%s >> gpurun_out/stock.tick; done ) &
TICK=$!
trap "kill $TICK" EXIT
timeout -k 10 1100 python -u benchmarks/stock_baselines.py --model resnet50 --batch 1024 --steps 10 --warmup 3 --no-find > gpurun_out/stock_rn50_b1024.json 2> gpurun_out/stock_rn50_b1024.err
rc=$?
tail -5 gpurun_out/stock_rn50_b1024.err
cat gpurun_out/stock_rn50_b1024.json
exit $rc
