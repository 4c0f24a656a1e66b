#!/bin/bash
# GPU job (round 3 re-entry checkpoint): the whole -m gpu suite, smoke(), the headline bench, a steady-state
# rocprofv3 kernel trace of the bench (ResNet-50 b1024).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/ck_suite.log 2>&1 || { tail -60 gpurun_out/ck_suite.log; exit 1; }
tail -1 gpurun_out/ck_suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ck_smoke.log 2>&1 || { tail -20 gpurun_out/ck_smoke.log; exit 1; }
tail -1 gpurun_out/ck_smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/ck_bench.json 2> gpurun_out/ck_bench.err || { tail -30 gpurun_out/ck_bench.err; exit 1; }
cut -c1-300 gpurun_out/ck_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ck_prof -o rn -- python3 bench.py --steps 6 --warmup 2 > gpurun_out/ck_prof.log 2>&1 || { tail -20 gpurun_out/ck_prof.log; exit 1; }
grep '^{' gpurun_out/ck_prof.log | cut -c1-160
