#!/bin/bash
# Round-end check: default bench (seeded autotune, batch 1024), smoke.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/final
export TMPDIR=/tmp
K8S_AMD_AUTOTUNE_VERBOSE=1 timeout -k 10 600 python bench.py > gpurun_out/final/bench.log 2> gpurun_out/final/bench.err || { tail -20 gpurun_out/final/bench.err; exit 1; }
cat gpurun_out/final/bench.log
grep -c "^autotune .* -> " gpurun_out/final/bench.err || true
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/final/smoke.log 2>&1 && tail -1 gpurun_out/final/smoke.log
