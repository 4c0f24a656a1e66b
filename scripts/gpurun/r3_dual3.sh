#!/bin/bash
# GPU job (round 3): dual BN backward (one reduce sweep + one apply for bn3 and the downsample BN): ResNet GPU tests,
# then the headline bench A/B K8S_AMD_BN_DUAL_BWD=1 / 0 alternated.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_resnet_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/dual_tests.log 2>&1 || { grep -E "Error|assert" gpurun_out/dual_tests.log | cut -c1-3000 | tail -8; exit 1; }
tail -1 gpurun_out/dual_tests.log
bash scripts/gpurun/env_ab.sh "K8S_AMD_BN_DUAL_BWD=1" "K8S_AMD_BN_DUAL_BWD=0"
