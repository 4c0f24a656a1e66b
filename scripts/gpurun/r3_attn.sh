#!/bin/bash
# GPU job (round 3): flash attention numerics (both forward forms) and the kernel microbenchmark, A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1 || { tail -40 gpurun_out/attn_tests.log; exit 1; }
tail -1 gpurun_out/attn_tests.log
K8S_AMD_FA_FWD32=0 timeout -k 10 200 python -u scripts/bench_attention.py > gpurun_out/attn_bench_old.jsonl 2> gpurun_out/attn_bench_old.err || { tail -20 gpurun_out/attn_bench_old.err; exit 1; }
timeout -k 10 200 python -u scripts/bench_attention.py > gpurun_out/attn_bench_new.jsonl 2> gpurun_out/attn_bench_new.err || { tail -20 gpurun_out/attn_bench_new.err; exit 1; }
paste -d'\n' gpurun_out/attn_bench_old.jsonl gpurun_out/attn_bench_new.jsonl | cut -c1-230
timeout -k 10 300 python -u -m pytest tests/test_gemm_conv_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_gemm_tests.log 2>&1 || { tail -40 gpurun_out/attn_gemm_tests.log; exit 1; }
tail -1 gpurun_out/attn_gemm_tests.log
