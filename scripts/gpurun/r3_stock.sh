#!/bin/bash
# GPU job (round 3): stock PyTorch-ROCm baselines on the same MI355X: Llama-3-8B s4096 b1,
# Llama-1B s2048 b2, BERT-base (HF every-token MLM head) b64 s128, ResNet-50 b1024 with MIOpen's FAST find mode.
set -o pipefail
mkdir -p gpurun_out/stock
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/stock/$name.json 2> gpurun_out/stock/$name.err
  local rc=$?
  echo "$name rc=$rc $(grep '^{' gpurun_out/stock/$name.json | tail -1 | cut -c1-300)"
  return $rc
}
run llama3_8b 600 python -u benchmarks/stock_baselines.py --model llama3_8b --batch 1 --seq 4096 --steps 5 --warmup 2 &&
run llama_1b 300 python -u benchmarks/stock_baselines.py --model llama_1b --batch 2 --seq 2048 --steps 10 --warmup 3 &&
run bert_base 300 python -u benchmarks/stock_baselines.py --model bert_base --batch 64 --seq 128 --steps 20 --warmup 5 &&
run resnet50_fast 700 python -u benchmarks/stock_baselines.py --model resnet50 --batch 1024 --steps 10 --warmup 3 --miopen-find-mode FAST
