#!/bin/bash
# GPU job (round 5): 4-wave GEMM stagger (sleeper blocks delay half the CUs' first tile so the store-bound epilogues
# of the two halves stop coinciding) -- GEMM tests with it on, BERT GEMM microbench and BERT b1024 trainer A/B over
# K8S_AMD_G4_STAGGER (sleep loops of ~3.4 us).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_stagger; rm -rf $O; mkdir -p $O
K8S_AMD_G4_STAGGER=4 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm256_gpu.py tests/test_attention_gpu.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for v in 0 4 2 6 0 4; do
  K8S_AMD_G4_STAGGER=$v timeout -k 10 200 python -u scripts/bench_bert_gemm.py > $O/gemm_$v.jsonl 2>&1 || { tail -20 $O/gemm_$v.jsonl; exit 1; }
  echo "stagger=$v: $(python3 -c "import json,sys; print(' '.join('%s/%s %.0f' % (r['layer'], r['form'], r['us']) for r in (json.loads(l) for l in open(sys.argv[1]) if l.startswith('{'))))" $O/gemm_$v.jsonl)"
done
for v in 0 2 4 6 0 4; do
  K8S_AMD_G4_STAGGER=$v timeout -k 10 300 python -u -m k8s_amd.trainer --model bert_base --seq 128 --steps 40 --log-every 20 > $O/bert_$v.log 2>&1 || { tail -20 $O/bert_$v.log; exit 1; }
  echo "bert b1024 stagger=$v: $(grep '"event": "step"' $O/bert_$v.log | tail -1 | cut -c1-120)"
done
