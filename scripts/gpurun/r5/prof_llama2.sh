#!/bin/bash
# GPU job (round 5): Llama-3-8B b4 s4096 step profile, per (kernel, grid) for the GEMMs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_prof_llama2; rm -rf $O; mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/pl -o ll -- python3 -m k8s_amd.trainer --model llama3_8b --seq 4096 --steps 4 --log-every 2 --max-grad-norm 1.0 > $O/pl.log 2>&1 || { tail -20 $O/pl.log; exit 1; }
python3 scripts/grid_report.py $(ls $O/pl/*kernel_trace.csv | head -1) --match "" --step-marker adam_kernel > $O/llama_grid.txt && head -40 $O/llama_grid.txt
rm -rf $O/pl
