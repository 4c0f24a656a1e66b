#!/bin/bash
# GPU job (end of round 2): final_check.sh, then BERT-base throughput and its steady-state trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpurun/final_check.sh || exit 1
rm -rf gpurun_out/prof_bert
timeout -k 10 300 python -m k8s_amd.trainer --model bert_base --batch 64 --seq 128 --steps 30 --log-every 10 > gpurun_out/train_bert.log 2>&1 && grep '"step"' gpurun_out/train_bert.log | tail -1 | cut -c1-160 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bert -o bert -- python3 -m k8s_amd.trainer --model bert_base --batch 64 --seq 128 --steps 8 --log-every 4 > gpurun_out/prof_bert.log 2>&1 && echo bert prof ok
