#!/bin/bash
# GPU job (round 4): short-K GEMM ablation (stores off) on the ResNet-50 1x1 shapes.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/gpurun/r4/c1x1.py > gpurun_out/r4_gsk_abl0.jsonl 2> gpurun_out/r4_gsk_abl.err || { tail -30 gpurun_out/r4_gsk_abl.err; exit 1; }
K8S_AMD_GSK_ABL=1 timeout -k 10 300 python -u scripts/gpurun/r4/c1x1.py > gpurun_out/r4_gsk_abl1.jsonl 2>> gpurun_out/r4_gsk_abl.err || { tail -30 gpurun_out/r4_gsk_abl.err; exit 1; }
cat gpurun_out/r4_gsk_abl0.jsonl gpurun_out/r4_gsk_abl1.jsonl
