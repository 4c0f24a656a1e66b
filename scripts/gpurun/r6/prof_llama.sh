#!/bin/bash
# GPU job (round 6): Llama-3-8B b4 s4096 step profile per (kernel, grid), SwiGLU / RoPE epilogues on and off.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_prof_llama; rm -rf $O; mkdir -p $O
for v in 1 0; do
  K8S_AMD_SWIGLU_EPI=$v K8S_AMD_ROPE_EPI=$v timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/pl$v -o ll -- python3 -m k8s_amd.trainer --model llama3_8b --seq 4096 --steps 4 --log-every 2 --max-grad-norm 1.0 > $O/pl$v.log 2>&1 || { tail -20 $O/pl$v.log; exit 1; }
  python3 scripts/grid_report.py $(ls $O/pl$v/*kernel_trace.csv | head -1) --match "" --step-marker adam_kernel > $O/llama_grid_$v.txt && head -32 $O/llama_grid_$v.txt
  rm -rf $O/pl$v
done
