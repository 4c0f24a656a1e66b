#!/bin/bash
# GPU job: activation / attention / transformer tests, trainer throughput (BERT-base, Llama-3-8B), then
# steady-state kernel traces of both.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_bert gpurun_out/prof_llama8b
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_conv_gpu.py tests/test_kernels_gpu.py tests/test_transformer_grads_gpu.py > gpurun_out/act_test.log 2>&1 || { tail -40 gpurun_out/act_test.log; exit 1; }
tail -1 gpurun_out/act_test.log
timeout -k 10 300 python -m k8s_amd.trainer --model bert_base --batch 64 --seq 128 --steps 30 --log-every 10 > gpurun_out/train_bert.log 2>&1 && grep '"step"' gpurun_out/train_bert.log | tail -1 | cut -c1-160 &&
timeout -k 10 500 python -m k8s_amd.trainer --model llama3_8b --batch 1 --seq 4096 --steps 8 --log-every 2 --max-grad-norm 1.0 > gpurun_out/train_llama8b.log 2>&1 && grep '"step"' gpurun_out/train_llama8b.log | tail -1 | cut -c1-160 &&
bash scripts/gpurun/prof_transformers.sh
