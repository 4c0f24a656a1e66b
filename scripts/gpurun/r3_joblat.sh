#!/bin/bash
# GPU job (round 3): the TfJob path (operator -> pod -> trainer) at the headline config: create -> step 0 latency and
# steady img/s, next to bench.py on the same box.
set -o pipefail
mkdir -p gpurun_out/ours
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/jl_bench.json 2> gpurun_out/jl_bench.err || { tail -20 gpurun_out/jl_bench.err; exit 1; }
cut -c1-200 gpurun_out/jl_bench.json
timeout -k 10 600 python -u benchmarks/job_latency.py --runs 3 --steps 30 --log-every 10 > gpurun_out/ours/job_latency.json 2> gpurun_out/ours/job_latency.err || { tail -20 gpurun_out/ours/job_latency.err; exit 1; }
tail -1 gpurun_out/ours/job_latency.json | cut -c1-600
