#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bert -o bert -- python3 -m k8s_amd.trainer --model bert_base --batch 64 --seq 128 --steps 8 --log-every 4 > gpurun_out/prof_bert.log 2>&1 && echo bert ok
