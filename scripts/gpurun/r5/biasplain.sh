#!/bin/bash
# GPU job (round 5): bias on the plain 4-wave instantiation -- GEMM tests, BERT b1024 products (with hipBLASLt as the
# box calibration), bias-only routing A/B, BERT trainer.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_biasplain; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm256_gpu.py tests/test_transformer_grads_gpu.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
for v in 1 0; do
  K8S_AMD_G4_BIAS_PLAIN=$v timeout -k 10 200 python -u scripts/bench_bert_gemm.py --blas > $O/gemm_$v.jsonl 2>&1 || { tail -20 $O/gemm_$v.jsonl; exit 1; }
  echo "bias_plain=$v: $(python3 -c "import json,sys; print(' '.join('%s/%s %.0f' % (r['layer'], r['form'], r['us']) for r in (json.loads(l) for l in open(sys.argv[1]) if l.startswith('{'))))" $O/gemm_$v.jsonl)"
done
for v in 1 0; do
  K8S_AMD_G4_BIAS_PLAIN=$v timeout -k 10 300 python -u -m k8s_amd.trainer --model bert_base --seq 128 --steps 40 --log-every 20 > $O/bert_$v.log 2>&1 || { tail -20 $O/bert_$v.log; exit 1; }
  echo "bert b1024 bias_plain=$v: $(grep '"event": "step"' $O/bert_$v.log | tail -1 | cut -c1-120)"
done
