#!/bin/bash
# GPU job (round 5): BERT-base s128 at batch 64 on the final tree (the earlier reference point of the BASELINE row)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_bert64; rm -rf $O; mkdir -p $O
for b in 64 1024; do
  timeout -k 10 300 python -u -m k8s_amd.trainer --model bert_base --seq 128 --batch $b --steps 60 --log-every 20 > $O/bert_$b.log 2>&1 || { tail -20 $O/bert_$b.log; exit 1; }
  echo "bert b$b: $(grep '"event": "step"' $O/bert_$b.log | tail -1 | cut -c1-120)"
done
