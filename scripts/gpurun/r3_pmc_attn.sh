#!/bin/bash
# rocprofv3 counter passes over the flash-attention kernels (each pass its own run, SQ <= 8 counters).
set -o pipefail
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_attn
mkdir -p gpurun_out/pmc_attn
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc_attn/p$i -o p$i -- python3 scripts/pmc_attention.py > gpurun_out/pmc_attn/p$i.log 2>&1 || { tail -20 gpurun_out/pmc_attn/p$i.log; exit 1; }
done
find gpurun_out/pmc_attn -name "*.csv" | head -20
