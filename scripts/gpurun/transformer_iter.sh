#!/bin/bash
# GPU job: transformer tests (fp32-twin gradients, models, kernels), BERT-base throughput and a steady-state trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_transformer_grads_gpu.py tests/test_models_gpu.py tests/test_kernels_gpu.py tests/test_gemm_conv_gpu.py > gpurun_out/tr_test.log 2>&1 || { tail -40 gpurun_out/tr_test.log; exit 1; }
tail -2 gpurun_out/tr_test.log
timeout -k 10 300 python -m k8s_amd.trainer --model bert_base --batch 64 --seq 128 --steps 30 --log-every 10 > gpurun_out/train_bert.log 2>&1 && grep '"step"' gpurun_out/train_bert.log | tail -1 | cut -c1-200 &&
timeout -k 10 300 python -m k8s_amd.trainer --model llama_1b --batch 2 --seq 2048 --steps 20 --log-every 5 --max-grad-norm 1.0 > gpurun_out/train_llama1b.log 2>&1 && grep '"step"' gpurun_out/train_llama1b.log | tail -1 | cut -c1-200 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bert -o bert -- python3 -m k8s_amd.trainer --model bert_base --batch 64 --seq 128 --steps 8 --log-every 4 > gpurun_out/prof_bert.log 2>&1
echo "prof rc=$?"
