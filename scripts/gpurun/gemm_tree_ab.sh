#!/bin/bash
# GPU job: gemm256 tests, then bench_gemm256 (Llama products) in this tree and in abtest/old, alternated.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm256_gpu.py > gpurun_out/g256_test.log 2>&1 || { tail -30 gpurun_out/g256_test.log; exit 1; }
tail -1 gpurun_out/g256_test.log
for arm in new old new old; do
  if [ $arm = new ]; then dir=.; else dir=abtest/old; fi
  ( cd $dir && timeout -k 10 300 python -u scripts/bench_gemm256.py --only llama --rounds 2 2> /tmp/g.err ) > gpurun_out/g_$arm.jsonl || { tail -5 /tmp/g.err; exit 1; }
  python3 -c "
import json,sys
rs=[json.loads(l) for l in open('gpurun_out/g_$arm.jsonl')]
print('$arm', ' '.join('%s/%s=%d'%(r['layer'],r['form'][0],r['ours_tf']) for r in rs))"
done
