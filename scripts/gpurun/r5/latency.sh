#!/bin/bash
# GPU job (round 5): headline bench, then the TfJob path on the same box: create -> step 0 split and the
# trainer's steady-state rate.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_latency; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-200 $O/bench.json
timeout -k 10 600 python -u benchmarks/job_latency.py --runs ${RUNS:-3} --steps 30 --log-every 10 > $O/latency.json 2> $O/latency.err || { tail -30 $O/latency.err; exit 1; }
cat $O/latency.err | tail -5
cut -c1-700 $O/latency.json
