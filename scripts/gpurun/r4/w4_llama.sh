#!/bin/bash
# GPU job (round 4): 4-wave NT GEMM in the Llama-3-8B step -- gemm tests, throughput and a steady-state trace.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4_tf; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm256_gpu.py -x -q --timeout 120 --timeout-method thread > $O/g256w4_tests.log 2>&1 || { tail -30 $O/g256w4_tests.log; exit 1; }
tail -1 $O/g256w4_tests.log
timeout -k 10 600 python -u -m k8s_amd.trainer --model llama3_8b --batch 1 --seq 4096 --steps 12 --log-every 4 --max-grad-norm 1.0 > $O/llama3_8b_w4.log 2>&1 || { tail -20 $O/llama3_8b_w4.log; exit 1; }
grep '"event": "step"' $O/llama3_8b_w4.log | tail -1 | cut -c1-140
timeout -k 10 300 python -u -m k8s_amd.trainer --model llama_1b --batch 2 --seq 2048 --steps 30 --log-every 10 > $O/llama_1b_w4.log 2>&1 || { tail -20 $O/llama_1b_w4.log; exit 1; }
grep '"event": "step"' $O/llama_1b_w4.log | tail -1 | cut -c1-140
rm -rf $O/prof_llama_w4
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/prof_llama_w4 -o ll -- python3 -m k8s_amd.trainer --model llama3_8b --batch 1 --seq 4096 --steps 6 --log-every 3 --max-grad-norm 1.0 > $O/prof_llama_w4.log 2>&1 || { tail -20 $O/prof_llama_w4.log; exit 1; }
python3 scripts/profile_report.py $(ls $O/prof_llama_w4/*kernel_trace.csv | head -1) --step-marker adam_kernel --title "Llama-3-8B s4096 b1, round 4 (4-wave NT GEMM)" > $O/llama_w4.md && head -28 $O/llama_w4.md
