#!/bin/bash
# GPU job (round 5): QKV bias gradient from the one-block attention backward; one-tile attention forward for
# Sk <= 128 (A/B via K8S_AMD_FA_ONE_TILE) -- attention tests, microbench, BERT b1024 A/B, BERT profile.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_fbias; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_attention_gpu.py tests/test_transformer_grads_gpu.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for v in 1 0; do
  K8S_AMD_FA_ONE_TILE=$v ATTN_CASES=bert_s128,bert_s128_b1024 timeout -k 10 200 python -u scripts/bench_attention.py > $O/attn_$v.jsonl 2>&1 || { tail -20 $O/attn_$v.jsonl; exit 1; }
  echo "one_tile=$v"; grep case $O/attn_$v.jsonl
done
for v in 1 0 1; do
  K8S_AMD_FA_ONE_TILE=$v timeout -k 10 300 python -u -m k8s_amd.trainer --model bert_base --seq 128 --steps 40 --log-every 20 > $O/bert_$v.log 2>&1 || { tail -20 $O/bert_$v.log; exit 1; }
  echo "bert b1024 one_tile=$v: $(grep '"event": "step"' $O/bert_$v.log | tail -1 | cut -c1-120)"
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/pb -o bert -- python3 -m k8s_amd.trainer --model bert_base --seq 128 --steps 6 --log-every 3 > $O/pb.log 2>&1 || { tail -20 $O/pb.log; exit 1; }
python3 scripts/profile_report.py $(ls $O/pb/*kernel_trace.csv | head -1) --step-marker adam_kernel --top 30 --title "BERT-base s128 b1024, round 5 (one-block attention backward + QKV bias gradient, one-tile forward)" > $O/bert.md && head -4 $O/bert.md
rm -rf $O/pb
