#!/bin/bash
# GPU job (round 4): conflict-free staged-window conv3x3 -- tests vs fp32, A/B timing, PMC pass, headline bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/r4_pmc_c3b; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_conv3x3_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_c3b_tests.log 2>&1 || { tail -40 gpurun_out/r4_c3b_tests.log; exit 1; }
tail -2 gpurun_out/r4_c3b_tests.log
timeout -k 10 300 python -u scripts/bench_conv3x3.py > gpurun_out/r4_c3b_ab.jsonl 2> gpurun_out/r4_c3b_ab.err || { tail -30 gpurun_out/r4_c3b_ab.err; exit 1; }
cat gpurun_out/r4_c3b_ab.jsonl
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $O/p$i -o p -- python3 scripts/pmc_conv3x3.py > $O/p$i.log 2>&1 || { tail -20 $O/p$i.log; exit 1; }
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/r4_c3b_bench.json 2> gpurun_out/r4_c3b_bench.err || { tail -30 gpurun_out/r4_c3b_bench.err; exit 1; }
cut -c1-300 gpurun_out/r4_c3b_bench.json
