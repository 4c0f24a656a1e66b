#!/bin/bash
# GPU job (round 4): 4-wave NT GEMM with the fine MFMA interleave and buffer-load DMA -- tests, bench, one PMC pass.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm256_gpu.py -x -q --timeout 120 --timeout-method thread -k "w4 or stream_k or ragged" > gpurun_out/r4_w4c_tests.log 2>&1 || { tail -30 gpurun_out/r4_w4c_tests.log; exit 1; }
tail -1 gpurun_out/r4_w4c_tests.log
timeout -k 10 400 python -u scripts/bench_gemm256.py --rounds 5 --only llama > gpurun_out/r4_w4c.jsonl 2> gpurun_out/r4_w4c.err || { tail -30 gpurun_out/r4_w4c.err; exit 1; }
timeout -k 10 400 python -u scripts/bench_gemm256.py --rounds 5 --only square > gpurun_out/r4_w4c_sq.jsonl 2>> gpurun_out/r4_w4c.err || { tail -30 gpurun_out/r4_w4c.err; exit 1; }
python3 - <<'PY'
import json
for fn in ["gpurun_out/r4_w4c.jsonl", "gpurun_out/r4_w4c_sq.jsonl"]:
    for l in open(fn):
        r = json.loads(l)
        if r["form"] == "fwd":
            print("%-6s %-8s %-6s %6.1f us ours %5d TF  blas %5d TF  x%.3f" % (r["group"], r["layer"], r["form"], r["ours_us"], r["ours_tf"], r["blas_tf"], r["speedup"]))
PY
O=gpurun_out/r4_w4cpmc; rm -rf $O; mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
BV_SHAPE=4096,28672,4096 BV_FORM=fwd BV_WHO=ours timeout -s KILL 90 rocprofv3 --pmc $P1 --output-format csv -d $O/p1 -o p -- python3 scripts/blas_vs_ours.py > $O/p1.log 2>&1 || { tail -20 $O/p1.log; exit 1; }
BV_SHAPE=4096,28672,4096 BV_FORM=fwd BV_WHO=ours timeout -s KILL 90 rocprofv3 --pmc $P2 --output-format csv -d $O/p2 -o p -- python3 scripts/blas_vs_ours.py > $O/p2.log 2>&1 || { tail -20 $O/p2.log; exit 1; }
python3 scripts/pmc_summary.py $O/p1/p_counter_collection.csv $O/p2/p_counter_collection.csv --match gemm 2>&1 | grep "##\|->"
