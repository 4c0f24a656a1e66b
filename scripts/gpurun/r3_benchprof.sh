#!/bin/bash
# GPU job (round 3): smoke(), the headline bench (20 steps) and its steady-state rocprofv3 kernel trace.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/bp_prof
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/bp_smoke.log 2>&1 || { tail -20 gpurun_out/bp_smoke.log; exit 1; }
tail -1 gpurun_out/bp_smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bp_bench.json 2> gpurun_out/bp_bench.err || { tail -30 gpurun_out/bp_bench.err; exit 1; }
cut -c1-300 gpurun_out/bp_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bp_prof -o rn -- python3 bench.py --steps 6 --warmup 2 > gpurun_out/bp_prof.log 2>&1 || { tail -20 gpurun_out/bp_prof.log; exit 1; }
grep '^{' gpurun_out/bp_prof.log | cut -c1-160
