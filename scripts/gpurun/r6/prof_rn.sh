#!/bin/bash
# GPU job (round 6): ResNet-50 b3072 step profile on the current tree + conv3x3 PMC passes.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r6_prof_rn}; rm -rf $O; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o rn -- python3 bench.py --steps 6 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/profile_report.py $(ls $O/prof/*kernel_trace.csv | head -1) --step-marker sgd_kernel --top 75 --title "ResNet-50 b3072, round 6 ${1:-}" > $O/rn.md && head -40 $O/rn.md
rm -rf $O/prof
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $O/p$i -o p -- python3 scripts/pmc_conv3x3.py > $O/p$i.log 2>&1 || { tail -20 $O/p$i.log; exit 1; }
done
python3 scripts/pmc_summary.py $O/p1/p_counter_collection.csv $O/p2/p_counter_collection.csv --match conv3x3 > $O/pmc_c3.txt 2>&1; tail -40 $O/pmc_c3.txt
