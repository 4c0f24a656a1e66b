#!/bin/bash
# A/B of the BN per-element kernels' loads per trip (K8S_AMD_BN_UNROLL=1/2/4): BN tests, HBM GB/s on the
# ResNet-50 b512 shapes, then the ResNet-50 bench per variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bn_ab
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_conv_gpu.py tests/test_resnet_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/bn_ab/pytest.log 2>&1 || { tail -30 gpurun_out/bn_ab/pytest.log; exit 1; }
tail -2 gpurun_out/bn_ab/pytest.log
for u in 1 2 4; do
  K8S_AMD_BN_UNROLL=$u BN_BATCH=512 timeout -k 10 180 python scripts/bench_bn.py > gpurun_out/bn_ab/bn_u$u.jsonl 2>&1 || exit 1
  echo "u=$u"; cat gpurun_out/bn_ab/bn_u$u.jsonl
done
for u in 1 4 2; do
  K8S_AMD_BN_UNROLL=$u timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bn_ab/bench_u$u.log 2>&1 || exit 1
  echo "bench u=$u $(grep metric gpurun_out/bn_ab/bench_u$u.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
