#!/bin/bash
# GPU job (round 5): bias-only 4-wave GEMM epilogue through the plain copy-out loop -- GEMM tests, BERT b1024 products
# (vs hipBLASLt) and the trainer.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_biascopy; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm256_gpu.py tests/test_transformer_grads_gpu.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 200 python -u scripts/bench_bert_gemm.py --blas > $O/gemm.jsonl 2>&1 || { tail -20 $O/gemm.jsonl; exit 1; }
python3 -c "import json,sys; print(' '.join('%s/%s %.0f' % (r['layer'], r['form'], r['us']) for r in (json.loads(l) for l in open(sys.argv[1]) if l.startswith('{'))))" $O/gemm.jsonl
for v in 1 2; do
  timeout -k 10 300 python -u -m k8s_amd.trainer --model bert_base --seq 128 --steps 40 --log-every 20 > $O/bert_$v.log 2>&1 || { tail -20 $O/bert_$v.log; exit 1; }
  echo "bert b1024 run $v: $(grep '"event": "step"' $O/bert_$v.log | tail -1 | cut -c1-120)"
done
