#!/bin/bash
# GPU job (round 4): transformer configs with the stream-K GEMM tail -- throughput runs, then steady-state kernel
# traces of Llama-3-8B s4096 b1 and BERT-base s128 b64.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4_tf
O=gpurun_out/r4_tf
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc $(grep -E '"event": "(step|done)"' $O/$name.log | tail -2 | cut -c1-260 | tr '\n' ' ')"
  return $rc
}
run bert 300 python -u -m k8s_amd.trainer --model bert_base --batch 64 --seq 128 --steps 40 --log-every 20 &&
run llama_1b 300 python -u -m k8s_amd.trainer --model llama_1b --batch 2 --seq 2048 --steps 30 --log-every 10 &&
run llama3_8b 600 python -u -m k8s_amd.trainer --model llama3_8b --batch 1 --seq 4096 --steps 12 --log-every 4 --max-grad-norm 1.0 &&
rm -rf $O/prof_llama $O/prof_bert &&
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/prof_llama -o ll -- python3 -m k8s_amd.trainer --model llama3_8b --batch 1 --seq 4096 --steps 6 --log-every 3 --max-grad-norm 1.0 > $O/prof_llama.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_bert -o bb -- python3 -m k8s_amd.trainer --model bert_base --batch 64 --seq 128 --steps 20 --log-every 10 > $O/prof_bert.log 2>&1 &&
python3 scripts/profile_report.py $(ls $O/prof_llama/*kernel_trace.csv | head -1) --step-marker adam_kernel --title "Llama-3-8B s4096 b1, round 4" > $O/llama.md &&
python3 scripts/profile_report.py $(ls $O/prof_bert/*kernel_trace.csv | head -1) --step-marker adam_kernel --title "BERT-base s128 b64, round 4" > $O/bert.md &&
head -16 $O/llama.md && head -16 $O/bert.md
