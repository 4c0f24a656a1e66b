#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_attention_gpu.py -x -q > gpurun_out/pytest_attn.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_attn.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_attention.py > gpurun_out/bench_attn.log 2>&1; rc=$?; cat gpurun_out/bench_attn.log
exit $rc
