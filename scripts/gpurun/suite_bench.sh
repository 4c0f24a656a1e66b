#!/bin/bash
# GPU job: the whole `-m gpu` suite, then the headline bench (stderr carries the conv path / GEMM fallback counters).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/suite.log 2>&1 || { tail -60 gpurun_out/suite.log; exit 1; }
tail -3 gpurun_out/suite.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err && cat gpurun_out/bench.json && grep -E "conv paths|gemm fallbacks" gpurun_out/bench.err
