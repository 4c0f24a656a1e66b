#!/bin/bash
# GPU job (round 4): 4-wave (one wave per SIMD, 128 x 128 per wave) NT GEMM vs the 8-wave ring vs hipBLASLt.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm256_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_w4_tests.log 2>&1 || { tail -40 gpurun_out/r4_w4_tests.log; exit 1; }
tail -2 gpurun_out/r4_w4_tests.log
timeout -k 10 400 python -u scripts/bench_gemm256.py --rounds 3 --only llama --forms fwd --variants K8S_AMD_G256_W4=0 > gpurun_out/r4_w4_llama.jsonl 2> gpurun_out/r4_w4_llama.err || { tail -30 gpurun_out/r4_w4_llama.err; exit 1; }
cut -c1-260 gpurun_out/r4_w4_llama.jsonl
