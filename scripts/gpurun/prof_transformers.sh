#!/bin/bash
# GPU job: steady-state kernel traces of BERT-base (b64 s128) and Llama-3-8B (b1 s4096).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bert -o bert -- python3 -m k8s_amd.trainer --model bert_base --batch 64 --seq 128 --steps 8 --log-every 4 > gpurun_out/prof_bert.log 2>&1 && echo bert ok &&
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_llama8b -o llama8b -- python3 -m k8s_amd.trainer --model llama3_8b --batch 1 --seq 4096 --steps 4 --log-every 2 --max-grad-norm 1.0 > gpurun_out/prof_llama8b.log 2>&1 && echo llama ok
