#!/bin/bash
# GPU job (round 4): ResNet-50 1x1-conv forward shapes, ours vs hipBLASLt.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/gpurun/r4/c1x1.py > gpurun_out/r4_c1x1.jsonl 2> gpurun_out/r4_c1x1.err || { tail -30 gpurun_out/r4_c1x1.err; exit 1; }
K8S_AMD_GEMM256=2 timeout -k 10 300 python -u scripts/gpurun/r4/c1x1.py > gpurun_out/r4_c1x1_g2.jsonl 2>> gpurun_out/r4_c1x1.err || { tail -30 gpurun_out/r4_c1x1.err; exit 1; }
cat gpurun_out/r4_c1x1.jsonl
cat gpurun_out/r4_c1x1_g2.jsonl
