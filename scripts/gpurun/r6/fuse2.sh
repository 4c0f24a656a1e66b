#!/bin/bash
# GPU job (round 6): SwiGLU (64-blocked, wave-local) / RoPE (pair-per-lane) epilogues -- tests, then the Llama-3-8B
# b4 step profile on / off and a trainer A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_fuse2; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm256_gpu.py tests/test_gemm_conv_gpu.py tests/test_transformer_grads_gpu.py tests/test_models_gpu.py tests/test_attention_gpu.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
bash scripts/gpurun/r6/prof_llama.sh
for v in 1 0 1 0; do
  K8S_AMD_SWIGLU_EPI=$v K8S_AMD_ROPE_EPI=$v timeout -k 10 600 python -u -m k8s_amd.trainer --model llama3_8b --seq 4096 --steps 8 --log-every 4 > $O/llama_$v.log 2>&1 || { tail -20 $O/llama_$v.log; exit 1; }
  echo "llama3_8b b4 epi(swiglu+rope)=$v: $(grep '"event": "step"' $O/llama_$v.log | tail -1 | cut -c1-160)"
done
