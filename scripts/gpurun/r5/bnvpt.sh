#!/bin/bash
# GPU job (round 5): BatchNorm apply pass with 1 / 2 / 4 vectors per thread (K8S_AMD_BN_VPT) -- BN / ResNet tests,
# ResNet-50 bench A/B alternating, per-kernel profile of the default.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_bnvpt; rm -rf $O; mkdir -p $O
for v in 2 4; do
  K8S_AMD_BN_VPT=$v timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_resnet_gpu.py > $O/test_$v.log 2>&1 || { tail -40 $O/test_$v.log; exit 1; }
  echo "vpt=$v tests: $(tail -1 $O/test_$v.log)"
done
for v in 1 2 4 1 2 4; do
  K8S_AMD_BN_VPT=$v timeout -k 10 300 python -u bench.py > $O/bench_$v.json 2> $O/bench_$v.err || { tail -20 $O/bench_$v.err; exit 1; }
  echo "vpt=$v: $(python3 -c "import json,sys; r=json.load(open(sys.argv[1])); print(r['value'], r['ms_per_step'])" $O/bench_$v.json)"
done
for v in 1 2 4; do
  K8S_AMD_BN_VPT=$v timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/p$v -o rn -- python3 bench.py --steps 4 --warmup 2 > $O/p$v.log 2>&1 || { tail -20 $O/p$v.log; exit 1; }
  python3 scripts/profile_report.py $(ls $O/p$v/*kernel_trace.csv | head -1) --step-marker sgd_kernel --top 75 --title "ResNet-50 b3072, BN apply $v vectors / thread" > $O/rn_$v.md && head -4 $O/rn_$v.md | tail -1 && grep "bn_apply_kernel\|bn_bwd_apply_kernel" $O/rn_$v.md
  rm -rf $O/p$v
done
