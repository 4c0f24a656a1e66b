#!/bin/bash
# Whole-step hipGraph: correctness test, then eager vs --graph throughput through the trainer.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_graph_gpu.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_graph.log 2>&1; rc=$?; tail -6 gpurun_out/pytest_graph.log; [ $rc -eq 0 ] || exit $rc
for m in "bert_base --batch 64 --seq 128 --steps 40 --log-every 10" \
         "llama_1b --batch 2 --seq 2048 --steps 20 --log-every 5" \
         "resnet50 --batch 256 --steps 20 --log-every 5"; do
  n=$(echo $m | cut -d' ' -f1)
  timeout -k 10 300 python -m k8s_amd.trainer --model $m > gpurun_out/g_eager_$n.log 2>&1 || exit 1
  echo "eager $n $(grep '"step"' gpurun_out/g_eager_$n.log | tail -1 | cut -c1-120)"
  timeout -k 10 300 python -m k8s_amd.trainer --model $m --graph > gpurun_out/g_graph_$n.log 2>&1 || exit 1
  echo "graph $n $(grep '"step"' gpurun_out/g_graph_$n.log | tail -1 | cut -c1-120)"
done
