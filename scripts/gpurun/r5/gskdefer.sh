#!/bin/bash
# GPU job (round 5): short-K GEMM with deferred copy-out stores (K8S_AMD_GSK_DEFER) -- gemm_short / ResNet GPU tests,
# ResNet-50 bench A/B alternating, per-kernel profiles of both arms.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_gskdefer; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_short_gpu.py tests/test_resnet_gpu.py -k "not side_stream" > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for v in 1 0 1 0; do
  K8S_AMD_GSK_DEFER=$v timeout -k 10 300 python -u bench.py > $O/bench_$v.json 2> $O/bench_$v.err || { tail -20 $O/bench_$v.err; exit 1; }
  echo "defer=$v: $(cut -c1-140 $O/bench_$v.json)"
done
for v in 1 0; do
  K8S_AMD_GSK_DEFER=$v timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/p$v -o rn -- python3 bench.py --steps 4 --warmup 2 > $O/p$v.log 2>&1 || { tail -20 $O/p$v.log; exit 1; }
  python3 scripts/profile_report.py $(ls $O/p$v/*kernel_trace.csv | head -1) --step-marker sgd_kernel --top 75 --title "ResNet-50 b3072, short-K GEMM deferred stores = $v" > $O/rn_$v.md && head -4 $O/rn_$v.md && grep gemm_short $O/rn_$v.md
  rm -rf $O/p$v
done
