#!/bin/bash
# GPU job (round 4): staged-window 3x3 conv -- kernel tests vs fp32, A/B timing at b1024, then the headline bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv3x3_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_c3_tests.log 2>&1 || { tail -40 gpurun_out/r4_c3_tests.log; exit 1; }
tail -2 gpurun_out/r4_c3_tests.log
timeout -k 10 300 python -u scripts/bench_conv3x3.py > gpurun_out/r4_c3_ab.jsonl 2> gpurun_out/r4_c3_ab.err || { tail -30 gpurun_out/r4_c3_ab.err; exit 1; }
cat gpurun_out/r4_c3_ab.jsonl
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/r4_c3_bench.json 2> gpurun_out/r4_c3_bench.err || { tail -30 gpurun_out/r4_c3_bench.err; exit 1; }
cut -c1-300 gpurun_out/r4_c3_bench.json
