#!/bin/bash
# GPU job: the tests touched this iteration, the ResNet-50 bench, then a Llama-3-8B kernel trace (4 steps) for the
# per-dispatch view (scripts/trace_context.py reads gpurun_out/prof_llama8b/*kernel_trace.csv afterwards).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_gemm_conv_gpu.py -k "grad_clip or maxpool or adam or sgd" > gpurun_out/iter_test.log 2>&1 || { tail -40 gpurun_out/iter_test.log; exit 1; }
tail -2 gpurun_out/iter_test.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_llama8b -o llama8b -- python3 -m k8s_amd.trainer --model llama3_8b --batch 1 --seq 4096 --steps 4 --log-every 2 --max-grad-norm 1.0 > gpurun_out/prof_llama8b.log 2>&1
echo "prof rc=$?"
grep '"step"' gpurun_out/prof_llama8b.log | tail -1 | cut -c1-200
