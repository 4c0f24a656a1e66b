#!/bin/bash
# GPU job (round 3): our configs 1/3/4 with the current kernels, the TfJob path's ResNet-50 rate, and stock
# ResNet-50 b1024 (MIOpen FAST find; a heartbeat file keeps the silent find from being taken for a hang).
set -o pipefail
mkdir -p gpurun_out/ours gpurun_out/stock
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) &
HB=$!
trap "kill $HB" EXIT
bash scripts/gpurun/r3_ours.sh || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/cmp_bench.json 2> gpurun_out/cmp_bench.err || { tail -20 gpurun_out/cmp_bench.err; exit 1; }
cut -c1-200 gpurun_out/cmp_bench.json
timeout -k 10 600 python -u benchmarks/stock_baselines.py --model resnet50 --batch 1024 --steps 10 --warmup 3 --miopen-find-mode FAST > gpurun_out/stock/resnet50_fast.json 2> gpurun_out/stock/resnet50_fast.err
echo "stock resnet rc=$? $(grep '^{' gpurun_out/stock/resnet50_fast.json | cut -c1-250)"
