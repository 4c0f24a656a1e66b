#!/bin/bash
# rocprofv3 counter passes over the memory-bound 1x1 convolutions (scripts/pmc_1x1.py), one pass per counter set.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc1
timeout -k 10 120 python3 scripts/pmc_1x1.py > gpurun_out/pmc1/time.log 2>&1 || { tail -20 gpurun_out/pmc1/time.log; exit 1; }
cat gpurun_out/pmc1/time.log
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_COUNT"
P3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc1/p$i -o p$i -- python3 scripts/pmc_1x1.py > gpurun_out/pmc1/p$i.log 2>&1 || { tail -20 gpurun_out/pmc1/p$i.log; exit 1; }
done
find gpurun_out/pmc1 -name "*counter_collection.csv" | head
