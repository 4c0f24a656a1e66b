#!/bin/bash
# rocprofv3 counter passes over one short-K conv case of scripts/conv_ab.py (PMC_ONLY=<case index>).
set -o pipefail
export TMPDIR=/tmp
CASE=${1:-3}
mkdir -p gpurun_out/pmcc
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_COUNT"
P3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  PMC_ONLY=$CASE timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmcc/p$i -o p$i -- python3 scripts/conv_ab.py > gpurun_out/pmcc/p$i.log 2>&1 || { tail -20 gpurun_out/pmcc/p$i.log; exit 1; }
done
find gpurun_out/pmcc -name "*counter_collection.csv" | head
