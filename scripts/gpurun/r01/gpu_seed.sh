#!/bin/bash
# Produce the MI355X autotune seed table (k8s_amd/ops/tuned/gfx950.json) from the shipped benchmark configs,
# recording each model's throughput on the way, then measure a cold node's trainer start -> step0 with the seed
# (fresh user cache, fresh MIOpen caches).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out /tmp/mio_seed /tmp/mio_cold
export TMPDIR=/tmp
AT=gpurun_out/autotune-gfx950.json
rm -f $AT
export K8S_AMD_AUTOTUNE_SEED=0
M="MIOPEN_USER_DB_PATH=/tmp/mio_seed MIOPEN_CUSTOM_CACHE_DIR=/tmp/mio_seed"
env $M K8S_AMD_AUTOTUNE_CACHE=$AT timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/seed_bench.log 2>&1 &&
grep metric gpurun_out/seed_bench.log &&
env $M K8S_AMD_AUTOTUNE_CACHE=$AT timeout -k 10 300 python -m k8s_amd.trainer --model bert_base --batch 64 --seq 128 \
  --steps 30 --log-every 10 > gpurun_out/seed_bert.log 2>&1 && grep '"step"' gpurun_out/seed_bert.log | tail -1 &&
env $M K8S_AMD_AUTOTUNE_CACHE=$AT timeout -k 10 300 python -m k8s_amd.trainer --model llama_1b --batch 2 --seq 2048 \
  --steps 20 --log-every 5 --max-grad-norm 1.0 > gpurun_out/seed_llama1b.log 2>&1 &&
grep '"step"' gpurun_out/seed_llama1b.log | tail -1 &&
env $M K8S_AMD_AUTOTUNE_CACHE=$AT timeout -k 10 400 python -m k8s_amd.trainer --model llama3_8b --batch 1 --seq 4096 \
  --steps 8 --log-every 2 --max-grad-norm 1.0 > gpurun_out/seed_llama8b.log 2>&1 &&
grep '"step"' gpurun_out/seed_llama8b.log | tail -1 &&
mkdir -p k8s_amd/ops/tuned && cp $AT k8s_amd/ops/tuned/gfx950.json &&
unset K8S_AMD_AUTOTUNE_SEED &&
MIOPEN_USER_DB_PATH=/tmp/mio_cold MIOPEN_CUSTOM_CACHE_DIR=/tmp/mio_cold K8S_AMD_AUTOTUNE_CACHE=/tmp/at_cold.json \
  timeout -k 10 300 python -m k8s_amd.trainer --model resnet50 --batch 256 --steps 2 --log-every 1 \
  > gpurun_out/cold_seeded.log 2>&1 && echo "cold_seeded $(grep '"step0"' gpurun_out/cold_seeded.log)"
