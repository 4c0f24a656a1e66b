#!/bin/bash
# GPU job: split-K cost-model A/B on the bench, then the read-only bandwidth study.
set -o pipefail
bash scripts/gpurun/env_ab.sh "" "K8S_AMD_SPLITK_OLD=1" || exit 1
timeout -k 10 120 ./scripts/microbench/read_bw 1.0 > gpurun_out/read_bw.jsonl 2>&1 || { tail -5 gpurun_out/read_bw.jsonl; exit 1; }
cat gpurun_out/read_bw.jsonl
