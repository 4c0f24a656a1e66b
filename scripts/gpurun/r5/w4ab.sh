#!/bin/bash
# GPU job (round 5): ResNet-50 bench A/B of the 4-wave kernel routing ($K8S_AMD_GEMM_W4) on one box, then a kernel
# trace of the BERT step kept per (kernel, grid) for the per-shape rates.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_w4ab; rm -rf $O; mkdir -p $O
for arm in 1 0 1 0; do
  K8S_AMD_GEMM_W4=$arm timeout -k 10 300 python -u bench.py > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  echo "w4=$arm: $(python -c "import json; d=json.load(open('$O/b.json')); print(d['value'], d['ms_per_step'])")"
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/pb -o bert -- python3 -m k8s_amd.trainer --model bert_base --seq 128 --steps 6 --log-every 3 > $O/pb.log 2>&1 || { tail -20 $O/pb.log; exit 1; }
python3 scripts/grid_report.py $(ls $O/pb/*kernel_trace.csv | head -1) --match gemm --step-marker adam_kernel > $O/bert_grid.txt && head -40 $O/bert_grid.txt
rm -rf $O/pb
