#!/bin/bash
# GPU job (round 5): stock PyTorch-ROCm transformers at the new presets' batches (same harness as round 3):
# HF BertForPreTraining s128 at 1024, LlamaForCausalLM (Llama-3-8B shape) s4096 at 2 and 4.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_stock_tf; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u benchmarks/stock_baselines.py --model bert_base --batch 1024 --seq 128 --steps 20 --warmup 5 > $O/bert.json 2> $O/bert.err || { tail -20 $O/bert.err; exit 1; }
cut -c1-300 $O/bert.json
for b in 2 4; do
  timeout -k 10 500 python -u benchmarks/stock_baselines.py --model llama3_8b --batch $b --seq 4096 --steps 8 --warmup 3 > $O/llama_b$b.json 2> $O/llama_b$b.err || { tail -5 $O/llama_b$b.err; echo "stock llama b$b failed"; continue; }
  cut -c1-300 $O/llama_b$b.json
done
