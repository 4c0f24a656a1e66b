#!/bin/bash
# GPU job: transformer correctness tests, then trainer throughput for BERT-base / Llama-1B / Llama-3-8B and a
# rocprofv3 kernel-trace summary of Llama-3-8B (every GEMM on our kernels: no vendor candidates).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_models_gpu.py tests/test_gemm256_gpu.py > gpurun_out/models_test.log 2>&1 || { tail -30 gpurun_out/models_test.log; exit 1; }
tail -2 gpurun_out/models_test.log
timeout -k 10 300 python -m k8s_amd.trainer --model bert_base --batch 64 --seq 128 --steps 30 --log-every 10 > gpurun_out/train_bert.log 2>&1 && grep '"step"' gpurun_out/train_bert.log | tail -1 | cut -c1-200 &&
timeout -k 10 300 python -m k8s_amd.trainer --model llama_1b --batch 2 --seq 2048 --steps 20 --log-every 5 --max-grad-norm 1.0 > gpurun_out/train_llama1b.log 2>&1 && grep '"step"' gpurun_out/train_llama1b.log | tail -1 | cut -c1-200 &&
timeout -k 10 500 python -m k8s_amd.trainer --model llama3_8b --batch 1 --seq 4096 --steps 8 --log-every 2 --max-grad-norm 1.0 > gpurun_out/train_llama8b.log 2>&1 && grep '"step"' gpurun_out/train_llama8b.log | tail -1 | cut -c1-200 &&
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_llama8b -o llama8b -- python3 -m k8s_amd.trainer --model llama3_8b --batch 1 --seq 4096 --steps 4 --log-every 2 --max-grad-norm 1.0 > gpurun_out/prof_llama8b.log 2>&1
echo "prof rc=$?"
