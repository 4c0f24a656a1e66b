#!/bin/bash
# GPU job (round 4): PMC of the 4-wave NT kernel against hipBLASLt on the gate_up forward (4096 x 28672 x 4096).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4_w4pmc
rm -rf $O; mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
P3="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum TCC_HIT_sum TCC_MISS_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  for who in ours blas; do
    BV_SHAPE=4096,28672,4096 BV_FORM=fwd BV_WHO=$who timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $O/${who}$i -o p -- python3 scripts/blas_vs_ours.py > $O/${who}$i.log 2>&1 || { tail -20 $O/${who}$i.log; echo "pass $i $who failed"; }
  done
done
for who in ours blas; do
  echo "== $who"
  python3 scripts/pmc_summary.py $O/${who}1/p_counter_collection.csv $O/${who}2/p_counter_collection.csv $O/${who}3/p_counter_collection.csv --match "gemm|Cijk" 2>&1 | grep -v "^  SQ_\|^  GRBM" | head -30
done
