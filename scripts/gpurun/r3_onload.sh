#!/bin/bash
# GPU job (round 3): normalize-on-load kernels' numerics, the ResNet gradient twin, then the bench with the BN apply
# passes of bn2 only / bn1 + bn2 / none normalised on load.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm_conv_gpu.py -k "normalize_on_load or bn_relu_conv" tests/test_resnet_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r3_onload.log 2>&1 || { tail -80 gpurun_out/r3_onload.log; exit 1; }
tail -3 gpurun_out/r3_onload.log
for mode in 1x1 all 0 1x1; do
  K8S_AMD_BN_ONLOAD=$mode timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r3_bench_$mode.json 2> gpurun_out/r3_bench_$mode.err || { tail -30 gpurun_out/r3_bench_$mode.err; exit 1; }
  echo "$mode $(cut -c1-200 gpurun_out/r3_bench_$mode.json)"
done
