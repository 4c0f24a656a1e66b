#!/bin/bash
# GPU job (round 3, end): steady-state rocprofv3 kernel trace of BERT-base (seq 128, batch 64) with the final kernels.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof_bert2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bert2 -o bb -- python3 -m k8s_amd.trainer --model bert_base --batch 64 --seq 128 --steps 20 --log-every 10 > gpurun_out/prof_bert2.log 2>&1 || { tail -20 gpurun_out/prof_bert2.log; exit 1; }
grep '"event": "step"' gpurun_out/prof_bert2.log | tail -1 | cut -c1-160
