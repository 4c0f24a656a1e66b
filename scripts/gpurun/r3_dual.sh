#!/bin/bash
# GPU job (round 3): downsample-block dual BN apply: headline bench A/B K8S_AMD_BN_DUAL=1 / 0 alternated, then the
# ResNet GPU tests (incl. fused vs separate against the fp32 twin).
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpurun/env_ab.sh "K8S_AMD_BN_DUAL=1" "K8S_AMD_BN_DUAL=0" || exit 1
timeout -k 10 400 python -u -m pytest tests/test_resnet_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/dual_tests.log 2>&1 || { grep -E "Error|assert" gpurun_out/dual_tests.log | cut -c1-3000 | tail -8; exit 1; }
tail -1 gpurun_out/dual_tests.log
