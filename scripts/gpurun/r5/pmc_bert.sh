#!/bin/bash
# GPU job (round 5): PMC of the BERT s128 attention kernels (one-block backward, one-tile forward) and the BERT b1024
# GEMM products vs hipBLASLt at training size.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_pmc_bert; rm -rf $O; mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  ATTN_SHAPE=bert timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $O/pa$i -o p -- python3 scripts/pmc_attention.py > $O/pa$i.log 2>&1 || { tail -20 $O/pa$i.log; exit 1; }
done
python3 scripts/pmc_summary.py $O/pa1/p_counter_collection.csv $O/pa2/p_counter_collection.csv --match flash > $O/attn_pmc.txt 2>&1 || true
grep -e "##" -e "MFMA busy" -e "per MFMA" -e "WAIT" -e "conflict" $O/attn_pmc.txt | head -40
timeout -k 10 300 python -u scripts/bench_bert_gemm.py --blas > $O/gemm.jsonl 2>&1 || { tail -20 $O/gemm.jsonl; exit 1; }
python3 -c "import json,sys; [print(r['layer'], r['form'], r['us'], r['tf']) for r in (json.loads(l) for l in open(sys.argv[1]) if l.startswith('{'))]" $O/gemm.jsonl
