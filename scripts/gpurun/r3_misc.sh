#!/bin/bash
# GPU job (round 3): MFMA shape microbenchmark, attention microbenchmark, Llama-3-8B / BERT steady-state profiles.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/microbench/mfma_shape > gpurun_out/mfma_shape.jsonl 2>&1 || { tail -5 gpurun_out/mfma_shape.jsonl; exit 1; }
cat gpurun_out/mfma_shape.jsonl
timeout -k 10 200 python -u scripts/bench_attention.py > gpurun_out/attn_bench_r3.jsonl 2> gpurun_out/attn_bench_r3.err || { tail -20 gpurun_out/attn_bench_r3.err; exit 1; }
rm -rf gpurun_out/prof_llama gpurun_out/prof_bert
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_llama -o ll -- python3 -m k8s_amd.trainer --model llama3_8b --batch 1 --seq 4096 --steps 6 --log-every 2 --max-grad-norm 1.0 > gpurun_out/prof_llama.log 2>&1 || { tail -20 gpurun_out/prof_llama.log; exit 1; }
grep '"event": "step"' gpurun_out/prof_llama.log | tail -1 | cut -c1-160
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bert -o bb -- python3 -m k8s_amd.trainer --model bert_base --batch 64 --seq 128 --steps 20 --log-every 10 > gpurun_out/prof_bert.log 2>&1 || { tail -20 gpurun_out/prof_bert.log; exit 1; }
grep '"event": "step"' gpurun_out/prof_bert.log | tail -1 | cut -c1-160
