#!/bin/bash
# GPU job: world-1 RCCL transports, the 2-rank gloo memory checks, the transformer/attention tests (linear_bwd /
# in-place rope guards), then the forced-RCCL bench record.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r6_rccl}; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread ${TESTS:-tests/test_rccl_gpu.py tests/test_dist_gpu.py} tests/test_transformer_grads_gpu.py tests/test_attention_gpu.py tests/test_models_gpu.py > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u bench.py --force-dist --grad-comm bf16 --steps 10 --warmup 3 > $O/bench_force.json 2> $O/bench_force.err || { tail -20 $O/bench_force.err; exit 1; }
cat $O/bench_force.json
