#!/bin/bash
# GPU job (round 4): 4-wave NT GEMM with the spread op schedule -- tests, transformer products vs hipBLASLt, the
# Llama-3-8B step (throughput + steady-state trace).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4_tf; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm256_gpu.py -x -q --timeout 120 --timeout-method thread > $O/g256f_tests.log 2>&1 || { tail -30 $O/g256f_tests.log; exit 1; }
tail -1 $O/g256f_tests.log
timeout -k 10 600 python -u scripts/bench_gemm256.py --rounds 5 > gpurun_out/r4_gemm_final.jsonl 2> gpurun_out/r4_gemm_final.err || { tail -30 gpurun_out/r4_gemm_final.err; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/r4_gemm_final.jsonl"):
    r = json.loads(l)
    print("%-6s %-8s %-6s %6.1f us ours %5d TF  blas %5d TF  x%.3f" % (r["group"], r["layer"], r["form"], r["ours_us"], r["ours_tf"], r["blas_tf"], r["speedup"]))
PY
timeout -k 10 600 python -u -m k8s_amd.trainer --model llama3_8b --batch 1 --seq 4096 --steps 12 --log-every 4 --max-grad-norm 1.0 > $O/llama3_8b_f.log 2>&1 || { tail -20 $O/llama3_8b_f.log; exit 1; }
grep '"event": "step"' $O/llama3_8b_f.log | tail -1 | cut -c1-140
rm -rf $O/prof_llama_f
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/prof_llama_f -o ll -- python3 -m k8s_amd.trainer --model llama3_8b --batch 1 --seq 4096 --steps 6 --log-every 3 --max-grad-norm 1.0 > $O/prof_llama_f.log 2>&1 || { tail -20 $O/prof_llama_f.log; exit 1; }
python3 scripts/profile_report.py $(ls $O/prof_llama_f/*kernel_trace.csv | head -1) --step-marker adam_kernel --title "Llama-3-8B s4096 b1, round 4 final" > $O/llama_f.md && head -24 $O/llama_f.md
