#!/bin/bash
# GPU job (round 6): whole GPU suite, smoke, bench at b3072 (default) and b1024.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r6_suite}; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/suite.log 2>&1 || { tail -40 $O/suite.log; exit 1; }
tail -1 $O/suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for b in 3072 1024 3072 1024; do
  timeout -k 10 400 python -u bench.py --batch $b > $O/bench_$b.json 2> $O/bench_$b.err || { tail -20 $O/bench_$b.err; exit 1; }
  python3 -c "import json,sys; r=json.load(open(sys.argv[1])); print('bench b%d' % r['config']['per_gpu_batch'], r['value'], r['ms_per_step'], r['peak_mem_gb'])" $O/bench_$b.json
done
