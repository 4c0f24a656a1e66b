#!/bin/bash
# GPU job (round 3): attention numerics + microbenchmark after the forward's unmasked/masked tile-loop split.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1 || { tail -40 gpurun_out/attn_tests.log; exit 1; }
tail -1 gpurun_out/attn_tests.log
timeout -k 10 200 python -u scripts/bench_attention.py > gpurun_out/attn_bench.jsonl 2> gpurun_out/attn_bench.err || { tail -20 gpurun_out/attn_bench.err; exit 1; }
cut -c1-260 gpurun_out/attn_bench.jsonl
