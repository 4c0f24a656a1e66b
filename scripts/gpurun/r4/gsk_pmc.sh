#!/bin/bash
# GPU job (round 4): PMC of the short-K streaming GEMM on two ResNet-50 shapes (HBM bytes, MFMA busy, waits).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4_gskpmc; rm -rf $O; mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
for c in fwd dgrad; do
  i=0
  for P in "$P1" "$P2" "$P3" "$P4"; do
    i=$((i+1))
    GSK_CASE=$c timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $O/${c}$i -o p -- python3 scripts/gpurun/r4/gsk_pmc.py > $O/${c}$i.log 2>&1 || { tail -20 $O/${c}$i.log; exit 1; }
  done
  echo "== $c"
  python3 scripts/pmc_summary.py $O/${c}1/p_counter_collection.csv $O/${c}2/p_counter_collection.csv $O/${c}3/p_counter_collection.csv $O/${c}4/p_counter_collection.csv --match "gemm_short" 2>&1 | head -40
done
