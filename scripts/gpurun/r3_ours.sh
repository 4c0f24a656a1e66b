#!/bin/bash
# GPU job (round 3): our trainer on the same configs as scripts/gpurun/r3_stock.sh, plus the TfJob path's
# ResNet-50 throughput and create -> step0 latency.
set -o pipefail
mkdir -p gpurun_out/ours
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/ours/$name.log 2> gpurun_out/ours/$name.err
  local rc=$?
  echo "$name rc=$rc $(grep -E '"event": "(step|done)"' gpurun_out/ours/$name.log | tail -2 | cut -c1-260 | tr '\n' ' ')"
  return $rc
}
run bert_every 300 python -u -m k8s_amd.trainer --model bert_base --batch 64 --seq 128 --steps 40 --log-every 10 --mlm-head every-token &&
run bert_gathered 300 python -u -m k8s_amd.trainer --model bert_base --batch 64 --seq 128 --steps 40 --log-every 10 &&
run llama_1b 300 python -u -m k8s_amd.trainer --model llama_1b --batch 2 --seq 2048 --steps 30 --log-every 10 &&
run llama3_8b 600 python -u -m k8s_amd.trainer --model llama3_8b --batch 1 --seq 4096 --steps 12 --log-every 4 --max-grad-norm 1.0 &&
timeout -k 10 600 python -u benchmarks/job_latency.py --runs 3 --steps 30 --log-every 10 > gpurun_out/ours/job_latency.json 2> gpurun_out/ours/job_latency.err &&
tail -1 gpurun_out/ours/job_latency.json | cut -c1-400
