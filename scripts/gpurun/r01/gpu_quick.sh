#!/bin/bash
# GPU session: all GPU tests, then the ResNet bench (+ profile) and the attention bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log; tail -25 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 && grep metric gpurun_out/bench.log &&
timeout -k 10 300 python scripts/bench_attention.py > gpurun_out/bench_attn.log 2>&1 && cat gpurun_out/bench_attn.log &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 5 --warmup 3 > gpurun_out/prof.log 2>&1 && echo prof ok
