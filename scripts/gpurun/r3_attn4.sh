#!/bin/bash
# GPU job (round 3): attention numerics + microbenchmark, then the Llama trainer configs that use the kernels.
set -o pipefail
mkdir -p gpurun_out/ours
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1 || { tail -40 gpurun_out/attn_tests.log; exit 1; }
tail -1 gpurun_out/attn_tests.log
timeout -k 10 200 python -u scripts/bench_attention.py > gpurun_out/attn_bench.jsonl 2> gpurun_out/attn_bench.err || { tail -20 gpurun_out/attn_bench.err; exit 1; }
cut -c1-260 gpurun_out/attn_bench.jsonl
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/ours/$name.log 2> gpurun_out/ours/$name.err
  local rc=$?
  echo "$name rc=$rc $(grep -E '"event": "(step|done)"' gpurun_out/ours/$name.log | tail -2 | cut -c1-260 | tr '\n' ' ')"
  return $rc
}
run llama_1b 300 python -u -m k8s_amd.trainer --model llama_1b --batch 2 --seq 2048 --steps 30 --log-every 10 &&
run llama3_8b 600 python -u -m k8s_amd.trainer --model llama3_8b --batch 1 --seq 4096 --steps 12 --log-every 4 --max-grad-norm 1.0
