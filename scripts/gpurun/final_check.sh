#!/bin/bash
# GPU job (end of round): the whole -m gpu suite, the driver's smoke(), the headline bench, TfJob create -> step 0.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/final_suite.log 2>&1 || { tail -60 gpurun_out/final_suite.log; exit 1; }
tail -1 gpurun_out/final_suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { tail -20 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err || { tail -30 gpurun_out/final_bench.err; exit 1; }
cut -c1-220 gpurun_out/final_bench.json
timeout -k 10 600 python -u benchmarks/job_latency.py --runs 3 > gpurun_out/job_latency.json 2> gpurun_out/job_latency.err || { tail -20 gpurun_out/job_latency.err; exit 1; }
cut -c1-400 gpurun_out/job_latency.json
