#!/bin/bash
# One gpurun session: GPU tests, smoke, 1-GPU bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit and steps are chained with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-20}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 ; echo "pytest exit $?" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 && cat gpurun_out/smoke.log | tail -2 &&
timeout -k 10 600 python bench.py --steps $STEPS --warmup 5 > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 5 --warmup 3 > gpurun_out/prof.log 2>&1 && echo prof ok
