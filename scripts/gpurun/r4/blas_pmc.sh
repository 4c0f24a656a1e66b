#!/bin/bash
# GPU job (round 4): which hipBLASLt kernels run each Llama / BERT product form, and PMC of ours vs theirs on the
# gate_up forward (4096 x 28672 x 4096, both operands K-major).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4_blas
rm -rf $O; mkdir -p $O
for spec in "4096,28672,4096 fwd" "4096,6144,4096 fwd" "4096,28672,4096 dgrad" "8192,768,3072 fwd" "8192,2304,768 fwd" "8192,3072,768 dgrad"; do
  set -- $spec
  tag=$(echo "$1_$2" | tr ',' 'x')
  BV_SHAPE=$1 BV_FORM=$2 BV_WHO=blas timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$tag -o kt -- python3 scripts/blas_vs_ours.py > $O/kt_$tag.log 2>&1 || { tail -20 $O/kt_$tag.log; exit 1; }
done
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
P3="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum TCC_HIT_sum TCC_MISS_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  BV_SHAPE=4096,28672,4096 BV_FORM=fwd timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $O/pmc$i -o p -- python3 scripts/blas_vs_ours.py > $O/pmc$i.log 2>&1 || { tail -20 $O/pmc$i.log; echo "pass $i failed"; }
done
find $O -name "*kernel_stats.csv" -o -name "*counter_collection.csv" | sort
