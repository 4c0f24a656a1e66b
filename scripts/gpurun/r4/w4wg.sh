#!/bin/bash
# GPU job (round 4): 4-wave NT GEMM for every operand layout (wgrad: fp32 out) -- gemm256 tests, the Llama products vs hipBLASLt.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm256_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_w4wg_tests.log 2>&1 || { tail -30 gpurun_out/r4_w4wg_tests.log; exit 1; }
tail -1 gpurun_out/r4_w4wg_tests.log
timeout -k 10 400 python -u scripts/bench_gemm256.py --rounds 5 --only llama > gpurun_out/r4_w4wg.jsonl 2> gpurun_out/r4_w4wg.err || { tail -30 gpurun_out/r4_w4wg.err; exit 1; }
K8S_AMD_GEMM_W4=0 timeout -k 10 400 python -u scripts/bench_gemm256.py --rounds 5 --only llama > gpurun_out/r4_w4wg_off.jsonl 2>> gpurun_out/r4_w4wg.err || { tail -30 gpurun_out/r4_w4wg.err; exit 1; }
python3 - <<'PY'
import json
for fn in ["gpurun_out/r4_w4wg.jsonl", "gpurun_out/r4_w4wg_off.jsonl"]:
    print(fn)
    for l in open(fn):
        r = json.loads(l)
        if True:
            print("%-6s %-8s %-6s %6.1f us ours %5d TF  blas %5d TF  x%.3f" % (r["group"], r["layer"], r["form"], r["ours_us"], r["ours_tf"], r["blas_tf"], r["speedup"]))
PY
