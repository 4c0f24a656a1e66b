#!/bin/bash
# GPU job: BatchNorm kernels' numerics + the ResNet gradient twin, then the bench A/B of the flat backward reduce.
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "bn" tests/test_resnet_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3_bnflat.log 2>&1 || { tail -40 gpurun_out/r3_bnflat.log; exit 1; }
tail -1 gpurun_out/r3_bnflat.log
bash scripts/gpurun/env_ab.sh "" "K8S_AMD_BN_FLAT_REDUCE=0"
