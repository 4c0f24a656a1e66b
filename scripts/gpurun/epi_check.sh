#!/bin/bash
# GPU job: GEMM epilogue + transformer tests, ResNet bench A/B against abtest/old, BERT throughput.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_conv_gpu.py tests/test_transformer_grads_gpu.py tests/test_models_gpu.py > gpurun_out/ep_test.log 2>&1 || { tail -40 gpurun_out/ep_test.log; exit 1; }
tail -1 gpurun_out/ep_test.log
bash scripts/gpurun/tree_ab.sh &&
timeout -k 10 300 python -m k8s_amd.trainer --model bert_base --batch 64 --seq 128 --steps 30 --log-every 10 > gpurun_out/train_bert.log 2>&1 && grep '"step"' gpurun_out/train_bert.log | tail -1 | cut -c1-160
