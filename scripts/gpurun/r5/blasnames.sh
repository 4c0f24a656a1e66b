#!/bin/bash
# GPU job (round 5): which hipBLASLt kernels (macro tile, depth, workgroup) run the BERT b1024 forward products that
# beat the 4-wave kernel -- kernel trace of the microbench's hipBLASLt arms.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_blasnames; rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o k -- python3 scripts/bench_bert_gemm.py --blas --reps 3 > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/r5_blasnames/kt/*kernel_stats.csv")[0]
rows = list(csv.DictReader(open(f)))
for r in rows:
    n = r["Name"]
    if "Cijk" in n or "gemm" in n.lower():
        print(r["Calls"], r["AverageNs"], n[:400])
PY
python3 - <<'PY' > gpurun_out/r5_blasnames/grid.txt
import csv, glob
f = glob.glob("gpurun_out/r5_blasnames/kt/*kernel_trace.csv")[0]
seen = set()
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"]
    if "Cijk" not in n: continue
    key = (n, r.get("Grid_Size_X", r.get("Grid_Size", "")), r.get("Workgroup_Size_X", r.get("Workgroup_Size", "")), r.get("LDS_Block_Size", r.get("Lds_Size", "")), r.get("VGPR_Count", r.get("Arch_VGPR_Count", "")), r.get("Accum_VGPR_Count", ""))
    if key in seen: continue
    seen.add(key)
    print(key)
PY
cat gpurun_out/r5_blasnames/grid.txt
rm -rf $O/kt
