#!/bin/bash
# GPU job (round 5): LayerNorm parameter-gradient partials folded in two levels -- norm / transformer tests, BERT b1024
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_normfold; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_transformer_grads_gpu.py tests/test_attention_gpu.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for v in 1 2; do
  timeout -k 10 300 python -u -m k8s_amd.trainer --model bert_base --seq 128 --steps 40 --log-every 20 > $O/bert_$v.log 2>&1 || { tail -20 $O/bert_$v.log; exit 1; }
  echo "bert b1024 run $v: $(grep '"event": "step"' $O/bert_$v.log | tail -1 | cut -c1-120)"
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/pb -o bert -- python3 -m k8s_amd.trainer --model bert_base --seq 128 --steps 6 --log-every 3 > $O/pb.log 2>&1 || { tail -20 $O/pb.log; exit 1; }
python3 scripts/profile_report.py $(ls $O/pb/*kernel_trace.csv | head -1) --step-marker adam_kernel --top 40 --title "BERT-base s128 b1024, round 5 (final)" > $O/bert.md && head -4 $O/bert.md && grep -e colsum -e norm_ $O/bert.md
rm -rf $O/pb
