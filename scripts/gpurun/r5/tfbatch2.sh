#!/bin/bash
# GPU job (round 5): BERT-base s128 at 512 / 1024 and Llama-3-8B s4096 at 2 / 4 per GPU, with peak memory.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_tfbatch2; rm -rf $O; mkdir -p $O
for b in 512 1024; do
  timeout -k 10 300 python -u -m k8s_amd.trainer --model bert_base --batch $b --seq 128 --steps 40 --log-every 20 > $O/bert_b$b.log 2>&1 || { tail -20 $O/bert_b$b.log; exit 1; }
  echo "bert b$b: $(grep '"event": "step"' $O/bert_b$b.log | tail -1 | cut -c1-110) $(grep -o '"peak_mem_gb": [0-9.]*' $O/bert_b$b.log)"
done
for b in 2 4; do
  timeout -k 10 500 python -u -m k8s_amd.trainer --model llama3_8b --batch $b --seq 4096 --steps 12 --log-every 4 --max-grad-norm 1.0 > $O/llama_b$b.log 2>&1 || { tail -5 $O/llama_b$b.log; echo "llama b$b failed"; continue; }
  echo "llama b$b: $(grep '"event": "step"' $O/llama_b$b.log | tail -1 | cut -c1-110) $(grep -o '"peak_mem_gb": [0-9.]*' $O/llama_b$b.log)"
done
