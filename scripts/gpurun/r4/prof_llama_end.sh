#!/bin/bash
# GPU job (round 4 end): Llama-3-8B s4096 steady-state kernel trace on the final tree.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4_llama_end; rm -rf $O; mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o ll -- python3 -m k8s_amd.trainer --model llama3_8b --batch 1 --seq 4096 --steps 6 --log-every 3 --max-grad-norm 1.0 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/profile_report.py $(ls $O/prof/*kernel_trace.csv | head -1) --step-marker adam_kernel --title "Llama-3-8B s4096 b1, round 4 final tree" > $O/llama.md && head -24 $O/llama.md
