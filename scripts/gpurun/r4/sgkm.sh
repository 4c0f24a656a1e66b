#!/bin/bash
# GPU job (round 4): 1x1 strided data gradient's live parity on the K-major source vs ConvA (K8S_AMD_SUBGRID_KMAJOR).
set -o pipefail
O=gpurun_out/r4_sgkm; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_conv_gpu.py tests/test_resnet_gpu.py -x -q --timeout 120 --timeout-method thread -k "strided or resnet" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 1 0; do
  K8S_AMD_SUBGRID_KMAJOR=$v timeout -k 10 300 python -u scripts/layer_roofline.py --only dgrad > $O/roof_$v.jsonl 2>> $O/err || { tail -20 $O/err; exit 1; }
  grep "b0.down" $O/roof_$v.jsonl | cut -c1-120
done
for r in 1 2; do
  for v in 1 0; do
    K8S_AMD_SUBGRID_KMAJOR=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_${v}_$r.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
    echo "sgkm=$v $(python3 -c "import json;d=json.load(open('$O/bench_${v}_$r.json'));print(d['value'], d['ms_per_step'])")"
  done
done
