#!/bin/bash
# GPU job (round 4): the whole GPU test suite, smoke() and the default bench, as the driver runs them.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r4_suite.log 2>&1 || { tail -40 gpurun_out/r4_suite.log; exit 1; }
tail -2 gpurun_out/r4_suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke.log 2>&1 || { tail -20 gpurun_out/r4_smoke.log; exit 1; }
tail -3 gpurun_out/r4_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r4_bench_default.json 2> gpurun_out/r4_bench_default.err || { tail -20 gpurun_out/r4_bench_default.err; exit 1; }
cut -c1-400 gpurun_out/r4_bench_default.json
