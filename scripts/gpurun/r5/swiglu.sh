#!/bin/bash
# GPU job (round 5): Llama's SwiGLU backward fused into the down projection's data gradient -- kernel / model tests,
# Llama-3-8B b4 trainer A/B (nn.SWIGLU_FUSE via K8S_AMD_SWIGLU_FUSE), profile.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_swiglu; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm256_gpu.py tests/test_transformer_grads_gpu.py tests/test_models_gpu.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for v in 1 0 1; do
  K8S_AMD_SWIGLU_FUSE=$v timeout -k 10 600 python -u -m k8s_amd.trainer --model llama3_8b --seq 4096 --steps 8 --log-every 4 > $O/llama_$v.log 2>&1 || { tail -20 $O/llama_$v.log; exit 1; }
  echo "llama3_8b b4 fuse=$v: $(grep '"event": "step"' $O/llama_$v.log | tail -1 | cut -c1-140)"
done
