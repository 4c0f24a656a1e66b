#!/bin/bash
# GPU job (round 4 end): the transformer trainers still step on the final tree (BERT-base, Llama-1B shape, Llama-3-8B).
set -o pipefail
O=gpurun_out/r4_trainers; rm -rf $O; mkdir -p $O
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc $(grep -E '"event": "step"' $O/$name.log | tail -1 | cut -c1-160)"
  return $rc
}
run bert 300 python -u -m k8s_amd.trainer --model bert_base --batch 64 --seq 128 --steps 40 --log-every 20 &&
run llama_1b 300 python -u -m k8s_amd.trainer --model llama_1b --batch 2 --seq 2048 --steps 30 --log-every 10 &&
run llama3_8b 600 python -u -m k8s_amd.trainer --model llama3_8b --batch 1 --seq 4096 --steps 12 --log-every 4 --max-grad-norm 1.0
