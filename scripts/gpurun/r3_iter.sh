#!/bin/bash
# GPU job (round 3 iteration): conv / GEMM kernel numerics, the 1x1 timing + VALU counter pass, the bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc1
timeout -k 10 300 python -u -m pytest tests/test_gemm_conv_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3_iter_tests.log 2>&1 || { tail -40 gpurun_out/r3_iter_tests.log; exit 1; }
tail -1 gpurun_out/r3_iter_tests.log
timeout -k 10 120 python3 scripts/pmc_1x1.py > gpurun_out/pmc1/time.log 2>&1 || { tail -20 gpurun_out/pmc1/time.log; exit 1; }
cat gpurun_out/pmc1/time.log | grep -v amdgpu.ids
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAVE_CYCLES --output-format csv -d gpurun_out/pmc1/q -o q -- python3 scripts/pmc_1x1.py > gpurun_out/pmc1/q.log 2>&1 || { tail -20 gpurun_out/pmc1/q.log; exit 1; }
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r3_iter_bench.json 2> gpurun_out/r3_iter_bench.err || { tail -30 gpurun_out/r3_iter_bench.err; exit 1; }
cut -c1-200 gpurun_out/r3_iter_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_iter -o rn -- python3 bench.py --steps 6 --warmup 2 > gpurun_out/prof_iter.log 2>&1 || { tail -20 gpurun_out/prof_iter.log; exit 1; }
grep '^{' gpurun_out/prof_iter.log | cut -c1-120
