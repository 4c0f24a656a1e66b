#!/bin/bash
# GPU job: kernel tests, then BERT-base throughput and its steady-state trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_bert
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py > gpurun_out/emb_test.log 2>&1 || { tail -40 gpurun_out/emb_test.log; exit 1; }
tail -1 gpurun_out/emb_test.log
timeout -k 10 300 python -m k8s_amd.trainer --model bert_base --batch 64 --seq 128 --steps 30 --log-every 10 > gpurun_out/train_bert.log 2>&1 && grep '"step"' gpurun_out/train_bert.log | tail -1 | cut -c1-160 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bert -o bert -- python3 -m k8s_amd.trainer --model bert_base --batch 64 --seq 128 --steps 8 --log-every 4 > gpurun_out/prof_bert.log 2>&1 && echo bert prof ok
