#!/bin/bash
# Where does a cold node's trainer-start -> step0 time go? Autotune (our per-shape timing) vs MIOpen
# (find-db / kernel compilation). Four runs toggling which cache is warm; each prints step0.since_start.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
AT=gpurun_out/autotune-gfx950.json
rm -f $AT
run() {  # $1=label $2=autotune cache $3=miopen dir
  mkdir -p "$3"
  K8S_AMD_AUTOTUNE_CACHE=$2 MIOPEN_USER_DB_PATH=$3 MIOPEN_CUSTOM_CACHE_DIR=$3 timeout -k 10 400 \
    python -m k8s_amd.trainer --model resnet50 --batch 256 --steps 2 --log-every 1 > gpurun_out/cold_$1.log 2>&1 &&
  echo "$1 $(grep '"step0"' gpurun_out/cold_$1.log)"
}
run cold_all $AT /tmp/mio1 &&
run warm_autotune $AT /tmp/mio2 &&
run warm_miopen /tmp/at_fresh.json /tmp/mio1 &&
run warm_all $AT /tmp/mio1 &&
ls -la /tmp/mio1 && du -sh /tmp/mio1
