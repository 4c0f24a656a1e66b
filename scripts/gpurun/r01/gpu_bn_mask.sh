#!/bin/bash
# Packed ReLU mask for residual BatchNorm backward: kernel + model GPU tests, ResNet-50 bench b512/b256, profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/mask
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/mask/pytest.log 2>&1 || { tail -30 gpurun_out/mask/pytest.log; exit 1; }
tail -2 gpurun_out/mask/pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/mask/bench.log 2> gpurun_out/mask/bench.err || { tail -20 gpurun_out/mask/bench.err; exit 1; }
cat gpurun_out/mask/bench.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --batch 256 > gpurun_out/mask/bench256.log 2> gpurun_out/mask/bench256.err && cat gpurun_out/mask/bench256.log &&
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/mask/smoke.log 2>&1 && tail -1 gpurun_out/mask/smoke.log &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mask/prof -o run -- python bench.py --steps 5 --warmup 3 > gpurun_out/mask/prof.log 2>&1 && echo prof ok
