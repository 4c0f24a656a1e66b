#!/bin/bash
# GPU job (round 5): persistent 4-wave GEMM (one block per CU walking the tiles; the next tile's first two stages
# fetched while the copy-out stores drain) -- GEMM / transformer / ResNet GPU tests, BERT b1024 products and the
# trainer A/B over K8S_AMD_G4_PERSIST, Llama / square products.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_persist; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm256_gpu.py tests/test_transformer_grads_gpu.py tests/test_attention_gpu.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for v in 1 0; do
  K8S_AMD_G4_PERSIST=$v timeout -k 10 200 python -u scripts/bench_bert_gemm.py > $O/gemm_$v.jsonl 2>&1 || { tail -20 $O/gemm_$v.jsonl; exit 1; }
  echo "persist=$v: $(python3 -c "import json,sys; print(' '.join('%s/%s %.0f' % (r['layer'], r['form'], r['us']) for r in (json.loads(l) for l in open(sys.argv[1]) if l.startswith('{'))))" $O/gemm_$v.jsonl)"
done
for v in 1 0; do
  K8S_AMD_G4_PERSIST=$v timeout -k 10 300 python -u scripts/bench_gemm256.py --only llama --forms fwd,dgrad --rounds 3 > $O/llama_$v.jsonl 2>&1 || { tail -20 $O/llama_$v.jsonl; exit 1; }
  echo "llama persist=$v: $(python3 -c "import json,sys; print(' '.join('%s/%s %s' % (r['layer'], r['form'], r['ours_tf']) for r in (json.loads(l) for l in open(sys.argv[1]) if l.startswith('{'))))" $O/llama_$v.jsonl)"
done
for v in 1 0 1 0; do
  K8S_AMD_G4_PERSIST=$v timeout -k 10 300 python -u -m k8s_amd.trainer --model bert_base --seq 128 --steps 40 --log-every 20 > $O/bert_$v.log 2>&1 || { tail -20 $O/bert_$v.log; exit 1; }
  echo "bert b1024 persist=$v: $(grep '"event": "step"' $O/bert_$v.log | tail -1 | cut -c1-120)"
done
