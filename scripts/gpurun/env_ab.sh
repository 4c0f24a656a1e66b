#!/bin/bash
# GPU job: the headline bench under several environment settings, alternated twice in one session on one box.
#   bash scripts/gpurun/env_ab.sh "K8S_AMD_X=0" "K8S_AMD_X=1" ...     (an empty string = the defaults)
set -o pipefail
mkdir -p gpurun_out
for round in 1 2; do
  for setting in "$@"; do
    env $setting timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > /tmp/ab.json 2> /tmp/ab.err || { tail -5 /tmp/ab.err; exit 1; }
    echo "[$setting] $(python3 -c "import json;d=json.load(open('/tmp/ab.json'));print(d['value'], d['ms_per_step'])")"
  done
done
