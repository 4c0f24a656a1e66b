#!/bin/bash
# rocprofv3 counter passes over the 256 x 256 GEMM (each pass its own run, SQ <= 8 counters).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc/p$i -o p$i -- python3 scripts/pmc_gemm256.py > gpurun_out/pmc/p$i.log 2>&1 || { tail -20 gpurun_out/pmc/p$i.log; exit 1; }
done
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc/kt -o kt -- python3 scripts/pmc_gemm256.py > gpurun_out/pmc/kt.log 2>&1
find gpurun_out/pmc -name "*.csv" | head -20
