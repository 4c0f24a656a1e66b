#!/bin/bash
# GPU job (round 6): stock PyTorch-ROCm ResNet-50 at the bench's own batch (3072) with MIOpen FAST find +
# cudnn.benchmark (ratios at the same batch); a heartbeat file keeps the silent search alive.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_stock; mkdir -p $O
( while sleep 50; do date +%s >> $O/heartbeat.txt; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 1100 python -u benchmarks/stock_baselines.py --model resnet50 --batch 3072 --steps 10 --warmup 3 --miopen-find-mode FAST > $O/resnet50_b3072_fast.json 2> $O/resnet50_b3072_fast.err
rc=$?
tail -3 $O/resnet50_b3072_fast.err
cat $O/resnet50_b3072_fast.json
exit $rc
