#!/bin/bash
# GPU job (round 3, last): the whole -m gpu suite and smoke() on the final tree.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/last_suite.log 2>&1 || { tail -60 gpurun_out/last_suite.log; exit 1; }
tail -1 gpurun_out/last_suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/last_smoke.log 2>&1 || { tail -20 gpurun_out/last_smoke.log; exit 1; }
tail -1 gpurun_out/last_smoke.log
