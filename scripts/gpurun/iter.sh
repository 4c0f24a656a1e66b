#!/bin/bash
# GPU job for one kernel iteration: the named GPU tests, the per-layer roofline (optional op subset), the bench.
#   bash scripts/gpurun/iter.sh "<test files>" "<roofline ops or ->" [bench args]
set -o pipefail
mkdir -p gpurun_out
TESTS=${1:-tests/test_gemm_conv_gpu.py}
OPS=${2:-fwd,dgrad}
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread $TESTS > gpurun_out/iter_test.log 2>&1 || { tail -40 gpurun_out/iter_test.log; exit 1; }
tail -1 gpurun_out/iter_test.log
if [ "$OPS" != "-" ]; then
  timeout -k 10 600 python -u scripts/layer_roofline.py --only $OPS > gpurun_out/roofline.jsonl 2> gpurun_out/roofline.err || { tail -30 gpurun_out/roofline.err; exit 1; }
  tail -1 gpurun_out/roofline.jsonl
fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 ${3} > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
