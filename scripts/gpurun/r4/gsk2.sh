#!/bin/bash
# GPU job (round 4): short-K GEMM with the row-contiguous copy-out -- tests, 1x1 shapes (K = 64 routed too), bench A/B.
set -o pipefail
O=gpurun_out/r4_gsk2; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_short_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
K8S_AMD_GEMM_SHORT64=1 timeout -k 10 300 python -u -m pytest tests/test_gemm_conv_gpu.py tests/test_resnet_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests2.log 2>&1 || { tail -40 $O/tests2.log; exit 1; }
tail -1 $O/tests2.log
K8S_AMD_GEMM_SHORT64=1 timeout -k 10 300 python -u scripts/gpurun/r4/c1x1.py > $O/on.jsonl 2> $O/err || { tail -30 $O/err; exit 1; }
cat $O/on.jsonl
for r in 1 2; do
  for v in 1 0; do
    K8S_AMD_GEMM_SHORT64=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_${v}_$r.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
    echo "short64=$v $(python3 -c "import json;d=json.load(open('$O/bench_${v}_$r.json'));print(d['value'], d['ms_per_step'])")"
  done
done
