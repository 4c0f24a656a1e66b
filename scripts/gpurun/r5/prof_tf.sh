#!/bin/bash
# GPU job (round 5): steady-state step profiles of the transformer trainers at the new presets.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_prof_tf; rm -rf $O; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/pb -o bert -- python3 -m k8s_amd.trainer --model bert_base --seq 128 --steps 8 --log-every 4 > $O/pb.log 2>&1 || { tail -20 $O/pb.log; exit 1; }
python3 scripts/profile_report.py $(ls $O/pb/*kernel_trace.csv | head -1) --step-marker adam_kernel --top 30 --title "BERT-base s128 b1024 (trainer preset), round 5" > $O/bert.md && head -45 $O/bert.md
rm -rf $O/pb
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/pl -o ll -- python3 -m k8s_amd.trainer --model llama3_8b --seq 4096 --steps 5 --log-every 5 --max-grad-norm 1.0 > $O/pl.log 2>&1 || { tail -20 $O/pl.log; exit 1; }
python3 scripts/profile_report.py $(ls $O/pl/*kernel_trace.csv | head -1) --step-marker adam_kernel --top 30 --title "Llama-3-8B s4096 b4 (trainer preset), round 5" > $O/llama.md && head -45 $O/llama.md
rm -rf $O/pl
