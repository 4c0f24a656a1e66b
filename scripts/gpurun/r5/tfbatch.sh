#!/bin/bash
# GPU job (round 5): transformer trainers at larger per-GPU batches (288 GB HBM sizing): BERT-base s128 at
# 64 / 256 / 512 and Llama-3-8B s4096 at 1 / 2 -- steady-state tokens/s from the trainer's own step log.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_tfbatch; rm -rf $O; mkdir -p $O
for b in 64 256 512; do
  timeout -k 10 300 python -u -m k8s_amd.trainer --model bert_base --batch $b --seq 128 --steps 40 --log-every 20 > $O/bert_b$b.log 2>&1 || { tail -20 $O/bert_b$b.log; exit 1; }
  echo "bert b$b: $(grep '"event": "step"' $O/bert_b$b.log | tail -1 | cut -c1-150)"
done
for b in 1 2; do
  timeout -k 10 500 python -u -m k8s_amd.trainer --model llama3_8b --batch $b --seq 4096 --steps 12 --log-every 4 --max-grad-norm 1.0 > $O/llama_b$b.log 2>&1 || { tail -20 $O/llama_b$b.log; exit 1; }
  echo "llama b$b: $(grep '"event": "step"' $O/llama_b$b.log | tail -1 | cut -c1-150)"
done
