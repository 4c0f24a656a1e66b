#!/bin/bash
# GPU job (round 4 start): GEMM vs hipBLASLt on every Llama-3-8B / BERT-base product, then the headline bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/bench_gemm256.py --rounds 3 > gpurun_out/r4_gemm_base.jsonl 2> gpurun_out/r4_gemm_base.err || { tail -30 gpurun_out/r4_gemm_base.err; exit 1; }
cat gpurun_out/r4_gemm_base.jsonl | cut -c1-220
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/r4_bench_base.json 2> gpurun_out/r4_bench_base.err || { tail -30 gpurun_out/r4_bench_base.err; exit 1; }
cut -c1-300 gpurun_out/r4_bench_base.json
