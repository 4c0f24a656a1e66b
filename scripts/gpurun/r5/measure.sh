#!/bin/bash
# GPU job (round 5): evidence refresh on the round-5 tree -- per-layer ResNet-50 roofline on the bench's code paths at
# the bench batch, the b3072 steady-state step profile, every transformer product vs hipBLASLt, attention PMC.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_measure; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u scripts/layer_roofline.py --batch ${BATCH:-3072} --reps 5 > $O/roof.jsonl 2> $O/roof.err || { tail -30 $O/roof.err; exit 1; }
tail -1 $O/roof.jsonl
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o rn -- python3 bench.py --steps 4 --warmup 2 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/profile_report.py $(ls $O/prof/*kernel_trace.csv | head -1) --step-marker sgd_kernel --top 75 --title "ResNet-50 b3072 (bench default), round 5" > $O/rn.md && head -14 $O/rn.md
rm -rf $O/prof
timeout -k 10 600 python -u scripts/bench_gemm256.py --rounds 5 > $O/gemm.jsonl 2> $O/gemm.err || { tail -30 $O/gemm.err; exit 1; }
python3 - <<'PY'
import json
rows = [json.loads(l) for l in open("gpurun_out/r5_measure/gemm.jsonl")]
print("gemm rows", len(rows), "below 0.95x:", sum(r["speedup"] < 0.95 for r in rows))
PY
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $O/pa$i -o p -- python3 scripts/pmc_attention.py > $O/pa$i.log 2>&1 || { tail -20 $O/pa$i.log; exit 1; }
done
python3 scripts/pmc_summary.py $O/pa1/p_counter_collection.csv $O/pa2/p_counter_collection.csv --match flash > $O/attn_pmc.txt 2>&1 || true
head -60 $O/attn_pmc.txt | grep -e "##" -e "MFMA busy" -e "per MFMA"
