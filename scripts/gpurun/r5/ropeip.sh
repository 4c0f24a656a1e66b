#!/bin/bash
# GPU job (round 5): Llama rotary embedding applied in place on the QKV projection output (no per-layer clone) --
# attention / model tests, Llama-3-8B b4 trainer.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_ropeip; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_attention_gpu.py tests/test_models_gpu.py tests/test_transformer_grads_gpu.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 600 python -u -m k8s_amd.trainer --model llama3_8b --seq 4096 --steps 8 --log-every 4 > $O/llama.log 2>&1 || { tail -20 $O/llama.log; exit 1; }
echo "llama3_8b b4: $(grep '"event": "step"' $O/llama.log | tail -1 | cut -c1-140)"
