#!/bin/bash
# GPU job (round 3): the Llama trainer configs (1B s2048 b2, 8B s4096 b1) with the current attention kernels.
set -o pipefail
mkdir -p gpurun_out/ours
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/ours/$name.log 2> gpurun_out/ours/$name.err
  local rc=$?
  echo "$name rc=$rc $(grep -E '"event": "(step|done)"' gpurun_out/ours/$name.log | tail -2 | cut -c1-260 | tr '\n' ' ')"
  return $rc
}
run llama_1b 300 python -u -m k8s_amd.trainer --model llama_1b --batch 2 --seq 2048 --steps 30 --log-every 10 &&
run llama3_8b 600 python -u -m k8s_amd.trainer --model llama3_8b --batch 1 --seq 4096 --steps 12 --log-every 4 --max-grad-norm 1.0 &&
run llama_1b_b 300 python -u -m k8s_amd.trainer --model llama_1b --batch 2 --seq 2048 --steps 30 --log-every 10 &&
run llama3_8b_b 600 python -u -m k8s_amd.trainer --model llama3_8b --batch 1 --seq 4096 --steps 12 --log-every 4 --max-grad-norm 1.0
