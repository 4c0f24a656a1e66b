#!/bin/bash
# GPU job: kernel + transformer-gradient tests, BERT-base trainer throughput, then a BERT-base kernel-trace profile.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_bert
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_transformer_grads_gpu.py > gpurun_out/bi_test.log 2>&1 || { tail -40 gpurun_out/bi_test.log; exit 1; }
tail -1 gpurun_out/bi_test.log
timeout -k 10 300 python -m k8s_amd.trainer --model bert_base --batch 64 --seq 128 --steps 30 --log-every 10 > gpurun_out/train_bert.log 2>&1 && grep '"step"' gpurun_out/train_bert.log | tail -2 | cut -c1-200 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bert -o bert -- python3 -m k8s_amd.trainer --model bert_base --batch 64 --seq 128 --steps 8 --log-every 4 > gpurun_out/prof_bert.log 2>&1 && echo bert prof ok
