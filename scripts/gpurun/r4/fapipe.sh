#!/bin/bash
# GPU job (round 4): software-pipelined D=64 flash-attention forward -- tests, then A/B against the unpipelined kernel.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_attention_gpu.py tests/test_transformer_grads_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4_fapipe_tests.log 2>&1 || { tail -30 gpurun_out/r4_fapipe_tests.log; exit 1; }
tail -1 gpurun_out/r4_fapipe_tests.log
rm -f gpurun_out/r4_fapipe.jsonl
for i in 1 2; do
  for p in 0 1; do
    echo "{\"pipe\": $p}" >> gpurun_out/r4_fapipe.jsonl
    K8S_AMD_FA_PIPE=$p timeout -k 10 200 python -u scripts/bench_attention.py >> gpurun_out/r4_fapipe.jsonl 2>> gpurun_out/r4_fapipe.err || { tail -20 gpurun_out/r4_fapipe.err; exit 1; }
  done
done
grep -v llama_s gpurun_out/r4_fapipe.jsonl | grep -v mha | cut -c1-160
