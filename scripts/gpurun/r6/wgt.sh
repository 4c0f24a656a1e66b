#!/bin/bash
# GPU job (round 6): wgrad_tile address rework -- tests, per-layer wgrad timings, bench x2, step profile.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_wgt; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_conv_gpu.py tests/test_conv3x3_gpu.py tests/test_planner_gpu.py tests/test_resnet_gpu.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 300 python -u scripts/layer_roofline.py --batch 3072 --reps 5 --only wgrad > $O/wgrad.jsonl 2> $O/wgrad.err || { tail -20 $O/wgrad.err; exit 1; }
grep conv2 $O/wgrad.jsonl | cut -c1-120
for i in 1 2; do
  timeout -k 10 300 python -u bench.py > $O/bench_$i.json 2> $O/bench_$i.err || { tail -20 $O/bench_$i.err; exit 1; }
  python3 -c "import json,sys; r=json.load(open(sys.argv[1])); print('bench', r['value'], r['ms_per_step'])" $O/bench_$i.json
done
bash scripts/gpurun/r6/prof_rn.sh r6_prof_wgt
