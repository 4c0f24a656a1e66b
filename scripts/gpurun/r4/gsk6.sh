#!/bin/bash
# GPU job (round 4): short-K GEMM, deferred epilogue for the K = 64 masked data gradient.
set -o pipefail
O=gpurun_out/r4_gsk6; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_short_gpu.py tests/test_gemm_conv_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u scripts/gpurun/r4/c1x1.py > $O/on.jsonl 2> $O/err || { tail -30 $O/err; exit 1; }
cut -c1-140 $O/on.jsonl
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_$r.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  echo "bench $(python3 -c "import json;d=json.load(open('$O/bench_$r.json'));print(d['value'], d['ms_per_step'])")"
done
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o rn -- python3 bench.py --steps 8 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/profile_report.py $(ls $O/prof/*kernel_trace.csv | head -1) --step-marker sgd_kernel --top 75 --title "ResNet-50 b1024, round 4 (deferred epilogue, K=64 masked dgrad)" > $O/rn.md && head -4 $O/rn.md && grep gemm_short $O/rn.md
