#!/bin/bash
# GPU job (round 3 checkpoint after the attention rework): the whole -m gpu suite, smoke(), the headline bench,
# steady-state rocprofv3 kernel traces of the bench (ResNet-50 b1024) and of Llama-3-8B s4096.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/fin_prof gpurun_out/fin_prof_llama
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/fin_suite.log 2>&1 || { tail -60 gpurun_out/fin_suite.log; exit 1; }
tail -1 gpurun_out/fin_suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin_smoke.log 2>&1 || { tail -20 gpurun_out/fin_smoke.log; exit 1; }
tail -1 gpurun_out/fin_smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/fin_bench.json 2> gpurun_out/fin_bench.err || { tail -30 gpurun_out/fin_bench.err; exit 1; }
cut -c1-300 gpurun_out/fin_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fin_prof -o rn -- python3 bench.py --steps 6 --warmup 2 > gpurun_out/fin_prof.log 2>&1 || { tail -20 gpurun_out/fin_prof.log; exit 1; }
grep '^{' gpurun_out/fin_prof.log | cut -c1-160
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fin_prof_llama -o ll -- python3 -m k8s_amd.trainer --model llama3_8b --batch 1 --seq 4096 --steps 6 --log-every 2 --max-grad-norm 1.0 > gpurun_out/fin_prof_llama.log 2>&1 || { tail -20 gpurun_out/fin_prof_llama.log; exit 1; }
grep '"done"' gpurun_out/fin_prof_llama.log | cut -c1-200
