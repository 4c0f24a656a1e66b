#!/bin/bash
# GPU job (round 4): every Llama-3-8B / BERT-base product, ours vs hipBLASLt, current code.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/bench_gemm256.py --rounds 5 > gpurun_out/r4_gemm_all.jsonl 2> gpurun_out/r4_gemm_all.err || { tail -30 gpurun_out/r4_gemm_all.err; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/r4_gemm_all.jsonl"):
    r = json.loads(l)
    print("%-6s %-8s %-6s %6.1f us ours %5d TF  blas %5d TF  x%.3f" % (r["group"], r["layer"], r["form"], r["ours_us"], r["ours_tf"], r["blas_tf"], r["speedup"]))
PY
