#!/bin/bash
# GPU job: TfJob create -> step 0 latency through the local cluster (cold box: fresh process, no MIOpen caches),
# then the stock PyTorch-ROCm ResNet-50 b1024 reference (MIOpen FAST find mode so its search fits the budget).
set -o pipefail
mkdir -p gpurun_out
( while sleep 50; do date +%s >> gpurun_out/evidence.tick; done ) &
TICK=$!
trap "kill $TICK" EXIT
timeout -k 10 600 python -u benchmarks/job_latency.py --runs 3 > gpurun_out/job_latency.json 2> gpurun_out/job_latency.err || { tail -20 gpurun_out/job_latency.err; exit 1; }
cat gpurun_out/job_latency.json
MIOPEN_FIND_MODE=FAST timeout -k 10 600 python -u benchmarks/stock_baselines.py --model resnet50 --batch 1024 --steps 10 --warmup 3 > gpurun_out/stock_rn50_b1024.json 2> gpurun_out/stock_rn50_b1024.err || { tail -20 gpurun_out/stock_rn50_b1024.err; exit 1; }
cat gpurun_out/stock_rn50_b1024.json
