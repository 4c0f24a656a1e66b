#!/bin/bash
# GPU job (round 4, end): GPU suite, smoke, ResNet bench, transformer steps and the Llama-3-8B steady-state trace.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4_final; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/suite.log 2>&1 || { tail -40 $O/suite.log; exit 1; }
tail -1 $O/suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-200 $O/bench.json
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc $(grep -E '"event": "step"' $O/$name.log | tail -1 | cut -c1-130)"
  return $rc
}
run bert 300 python -u -m k8s_amd.trainer --model bert_base --batch 64 --seq 128 --steps 40 --log-every 20 &&
run llama_1b 300 python -u -m k8s_amd.trainer --model llama_1b --batch 2 --seq 2048 --steps 30 --log-every 10 &&
run llama3_8b 600 python -u -m k8s_amd.trainer --model llama3_8b --batch 1 --seq 4096 --steps 12 --log-every 4 --max-grad-norm 1.0 || exit 1
rm -rf $O/prof_llama
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/prof_llama -o ll -- python3 -m k8s_amd.trainer --model llama3_8b --batch 1 --seq 4096 --steps 6 --log-every 3 --max-grad-norm 1.0 > $O/prof_llama.log 2>&1 || { tail -20 $O/prof_llama.log; exit 1; }
python3 scripts/profile_report.py $(ls $O/prof_llama/*kernel_trace.csv | head -1) --step-marker adam_kernel --title "Llama-3-8B s4096 b1, round 4 end (4-wave GEMM for all three forms)" > $O/llama.md && head -22 $O/llama.md
