#!/bin/bash
# GPU job: GEMM / conv / elementwise tests, headline bench x2 + its steady-state trace, transformer traces.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_conv_gpu.py > gpurun_out/late_test.log 2>&1 || { tail -40 gpurun_out/late_test.log; exit 1; }
tail -1 gpurun_out/late_test.log
bash scripts/gpurun/rn_final.sh && rm -rf gpurun_out/prof_bert gpurun_out/prof_llama8b && bash scripts/gpurun/prof_transformers.sh
