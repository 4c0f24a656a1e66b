#!/bin/bash
# GPU job (round 3, end): BERT-base throughput (every-token and gathered MLM heads) with the final kernels.
set -o pipefail
mkdir -p gpurun_out/ours
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/ours/$name.log 2> gpurun_out/ours/$name.err
  local rc=$?
  echo "$name rc=$rc $(grep -E '"event": "(step|done)"' gpurun_out/ours/$name.log | tail -2 | cut -c1-200 | tr '\n' ' ')"
  return $rc
}
run bert_every 300 python -u -m k8s_amd.trainer --model bert_base --batch 64 --seq 128 --steps 40 --log-every 10 --mlm-head every-token &&
run bert_gathered 300 python -u -m k8s_amd.trainer --model bert_base --batch 64 --seq 128 --steps 40 --log-every 10
