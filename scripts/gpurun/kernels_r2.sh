#!/bin/bash
# GPU job: GEMM / conv / streaming-wgrad correctness, then the wgrad and GEMM A/B benchmarks.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm256_gpu.py tests/test_wgrad_stream_gpu.py tests/test_gemm_conv_gpu.py > gpurun_out/kr2_test.log 2>&1 || { tail -40 gpurun_out/kr2_test.log; exit 1; }
tail -2 gpurun_out/kr2_test.log
timeout -k 10 400 python -u scripts/bench_wgrad.py > gpurun_out/bench_wgrad.jsonl 2> gpurun_out/bench_wgrad.err && cat gpurun_out/bench_wgrad.jsonl &&
timeout -k 10 400 python -u scripts/bench_gemm256.py --only square --rounds 3 > gpurun_out/gemm256_sq2.jsonl 2>&1 && cat gpurun_out/gemm256_sq2.jsonl
