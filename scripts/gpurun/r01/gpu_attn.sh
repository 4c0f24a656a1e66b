#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_attention.py > gpurun_out/bench_attn.log 2>&1; rc=$?; cat gpurun_out/bench_attn.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -m k8s_amd.trainer --model bert_base --batch 64 --seq 128 --steps 30 --log-every 10 \
  > gpurun_out/train_bert.log 2>&1 && grep '"step"' gpurun_out/train_bert.log | tail -1 &&
timeout -k 10 400 python -m k8s_amd.trainer --model llama_1b --batch 2 --seq 2048 --steps 20 --log-every 5 \
  --max-grad-norm 1.0 > gpurun_out/train_llama1b.log 2>&1 && grep '"step"' gpurun_out/train_llama1b.log | tail -1
