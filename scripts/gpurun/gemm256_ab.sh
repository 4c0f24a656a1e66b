#!/bin/bash
# GPU job: gemm256 A/B only (no tests): ring vs quad-phase variants vs hipBLASLt, args passed to the bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/bench_gemm256.py "$@" > gpurun_out/gemm256_bench.jsonl 2> gpurun_out/gemm256_bench.err
rc=$?
cat gpurun_out/gemm256_bench.jsonl
tail -5 gpurun_out/gemm256_bench.err
exit $rc
