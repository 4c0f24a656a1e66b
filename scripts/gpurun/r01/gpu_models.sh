#!/bin/bash
# GPU session: model throughput through the trainer (ours) and the TfJob create->step0 latency.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -m k8s_amd.trainer --model bert_base --batch 64 --seq 128 --steps 30 --log-every 10 \
  > gpurun_out/train_bert.log 2>&1 && grep '"step"' gpurun_out/train_bert.log | tail -1 &&
timeout -k 10 400 python -m k8s_amd.trainer --model llama_1b --batch 2 --seq 2048 --steps 20 --log-every 5 \
  --max-grad-norm 1.0 > gpurun_out/train_llama1b.log 2>&1 && grep '"step"' gpurun_out/train_llama1b.log | tail -1 &&
timeout -k 10 600 python -m k8s_amd.trainer --model llama3_8b --batch 1 --seq 4096 --steps 8 --log-every 2 \
  --max-grad-norm 1.0 > gpurun_out/train_llama8b.log 2>&1 && grep '"step"' gpurun_out/train_llama8b.log | tail -1 &&
timeout -k 10 600 python benchmarks/job_latency.py --runs 3 --steps 3 > gpurun_out/latency.log 2> gpurun_out/latency.err &&
tail -1 gpurun_out/latency.log
