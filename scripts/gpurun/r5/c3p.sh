#!/bin/bash
# GPU job (round 5): persistent pipelined 3x3 conv (c3p) -- tests, then the 3-arm timing A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_c3p; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_conv3x3_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u scripts/bench_conv3x3.py --rounds 3 > $O/bench.jsonl 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.jsonl
