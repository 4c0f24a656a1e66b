#!/bin/bash
# GPU job (round 4): stream-K tail of the 256 x 256 GEMM -- kernel tests, then Llama / BERT products vs hipBLASLt
# with the tail on and off (same process).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm256_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_sk_tests.log 2>&1 || { tail -40 gpurun_out/r4_sk_tests.log; exit 1; }
tail -2 gpurun_out/r4_sk_tests.log
timeout -k 10 400 python -u scripts/bench_gemm256.py --rounds 3 --only llama --variants K8S_AMD_GEMM256_SK=0 > gpurun_out/r4_sk_llama.jsonl 2> gpurun_out/r4_sk_llama.err || { tail -30 gpurun_out/r4_sk_llama.err; exit 1; }
cut -c1-260 gpurun_out/r4_sk_llama.jsonl
