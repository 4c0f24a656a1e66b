#!/bin/bash
# GPU job: max-pool tests, then the stem max-pool microbenchmark alternated between this tree and abtest/old.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_gemm_conv_gpu.py -k maxpool > gpurun_out/pool_test.log 2>&1 || { tail -40 gpurun_out/pool_test.log; exit 1; }
tail -1 gpurun_out/pool_test.log
for arm in new old new old; do
  if [ $arm = new ]; then dir=.; else dir=abtest/old; fi
  echo "$arm $( cd $dir && timeout -k 10 120 python -u scripts/bench_pool.py 2> /tmp/pool.err )" || { tail -5 /tmp/pool.err; exit 1; }
done
