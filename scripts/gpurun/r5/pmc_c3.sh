#!/bin/bash
# GPU job (round 5): PMC passes over the staged-window 3x3 conv at the three ResNet-50 stride-1 shapes.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_pmc_c3
rm -rf $O; mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $O/p$i -o p -- python3 scripts/pmc_conv3x3.py > $O/p$i.log 2>&1 || { tail -20 $O/p$i.log; exit 1; }
done
python3 scripts/pmc_summary.py $O/p1/p_counter_collection.csv $O/p2/p_counter_collection.csv --match conv3x3 2>&1 | tail -20 || true
