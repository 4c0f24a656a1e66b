#!/bin/bash
# GPU job (round 5): one-tile attention forward with 64-query blocks (K8S_AMD_FA_QS=1) vs 128 -- attention tests in
# both forms, microbench, BERT b1024 A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_faqs; rm -rf $O; mkdir -p $O
for v in 2 1; do
  K8S_AMD_FA_QS=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_attention_gpu.py > $O/test_$v.log 2>&1 || { tail -40 $O/test_$v.log; exit 1; }
  echo "qs=$v tests: $(tail -1 $O/test_$v.log)"
done
for v in 2 1; do
  K8S_AMD_FA_QS=$v ATTN_CASES=bert_s128,bert_s128_b1024 timeout -k 10 200 python -u scripts/bench_attention.py > $O/attn_$v.jsonl 2>&1 || { tail -20 $O/attn_$v.jsonl; exit 1; }
  echo "qs=$v"; grep case $O/attn_$v.jsonl | cut -c1-170
done
for v in 1 2 1 2; do
  K8S_AMD_FA_QS=$v timeout -k 10 300 python -u -m k8s_amd.trainer --model bert_base --seq 128 --steps 40 --log-every 20 > $O/bert_$v.log 2>&1 || { tail -20 $O/bert_$v.log; exit 1; }
  echo "bert b1024 qs=$v: $(grep '"event": "step"' $O/bert_$v.log | tail -1 | cut -c1-120)"
done
