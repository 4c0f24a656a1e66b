#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bert -o run -- python -m k8s_amd.trainer --model bert_base --batch 64 --seq 128 --steps 8 --log-every 4 > gpurun_out/prof_bert.log 2>&1 && echo bert ok &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_llama -o run -- python -m k8s_amd.trainer --model llama_1b --batch 2 --seq 2048 --steps 6 --log-every 3 > gpurun_out/prof_llama.log 2>&1 && echo llama ok
