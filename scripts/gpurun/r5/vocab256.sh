#!/bin/bash
# GPU job (round 5): BERT vocab padded to 256 columns (the MLM decoder on the 4-wave GEMM) -- transformer / model GPU
# tests, BERT b1024 trainer, per-kernel profile.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_vocab256; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_transformer_grads_gpu.py tests/test_models_gpu.py tests/test_kernels_gpu.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for v in 1 2; do
  timeout -k 10 300 python -u -m k8s_amd.trainer --model bert_base --seq 128 --steps 40 --log-every 20 > $O/bert_$v.log 2>&1 || { tail -20 $O/bert_$v.log; exit 1; }
  echo "bert b1024 run $v: $(grep '"event": "step"' $O/bert_$v.log | tail -1 | cut -c1-120)"
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/pb -o bert -- python3 -m k8s_amd.trainer --model bert_base --seq 128 --steps 6 --log-every 3 > $O/pb.log 2>&1 || { tail -20 $O/pb.log; exit 1; }
python3 scripts/profile_report.py $(ls $O/pb/*kernel_trace.csv | head -1) --step-marker adam_kernel --top 30 --title "BERT-base s128 b1024, round 5 (vocab padded to 256 columns)" > $O/bert.md && head -4 $O/bert.md
python3 scripts/grid_report.py $(ls $O/pb/*kernel_trace.csv | head -1) --match gemm --step-marker adam_kernel > $O/bert_grid.txt && head -16 $O/bert_grid.txt
rm -rf $O/pb
