#!/bin/bash
# GPU job (round 6): end-of-round BERT-base b1024 and Llama-3-8B b4 trainer runs on the final tree (regression check of
# the transformer configs next to the ResNet work).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_transformers; rm -rf $O; mkdir -p $O
timeout -k 10 500 python -u -m k8s_amd.trainer --model bert_base --seq 128 --steps 12 --log-every 4 > $O/bert.log 2>&1 || { tail -20 $O/bert.log; exit 1; }
echo "bert_base b1024: $(grep '"event": "step"' $O/bert.log | tail -1 | cut -c1-200)"
timeout -k 10 600 python -u -m k8s_amd.trainer --model llama3_8b --seq 4096 --steps 8 --log-every 4 > $O/llama.log 2>&1 || { tail -20 $O/llama.log; exit 1; }
echo "llama3_8b b4: $(grep '"event": "step"' $O/llama.log | tail -1 | cut -c1-200)"
