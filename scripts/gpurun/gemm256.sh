#!/bin/bash
# GPU job: gemm256 correctness tests, then the interleaved A/B vs hipBLASLt (args: extra bench flags).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm256_gpu.py > gpurun_out/gemm256_test.log 2>&1 || { tail -30 gpurun_out/gemm256_test.log; exit 1; }
tail -3 gpurun_out/gemm256_test.log
timeout -k 10 500 python -u scripts/bench_gemm256.py "$@" > gpurun_out/gemm256_bench.jsonl 2> gpurun_out/gemm256_bench.err
rc=$?
cat gpurun_out/gemm256_bench.jsonl
exit $rc
