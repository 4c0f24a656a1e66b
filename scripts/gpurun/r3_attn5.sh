#!/bin/bash
# GPU job (round 3): split dK/dV (chunked causal key blocks + fp32 partial reduce): numerics, then the attention
# microbenchmark with the default split rule and with K8S_AMD_FA_DKV_SPLIT=1 (unsplit) on the same box.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_attention_gpu.py tests/test_transformer_grads_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1 || { tail -40 gpurun_out/attn_tests.log; exit 1; }
tail -1 gpurun_out/attn_tests.log
timeout -k 10 200 python -u scripts/bench_attention.py > gpurun_out/attn_bench.jsonl 2> gpurun_out/attn_bench.err || { tail -20 gpurun_out/attn_bench.err; exit 1; }
K8S_AMD_FA_DKV_SPLIT=1 timeout -k 10 200 python -u scripts/bench_attention.py > gpurun_out/attn_bench_s1.jsonl 2> gpurun_out/attn_bench_s1.err || { tail -20 gpurun_out/attn_bench_s1.err; exit 1; }
paste -d'\n' gpurun_out/attn_bench.jsonl gpurun_out/attn_bench_s1.jsonl | cut -c1-220
