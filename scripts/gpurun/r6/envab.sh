#!/bin/bash
# Same-box A/B of environment switches on the default bench, arms alternating.
#   bash scripts/gpurun/r6/envab.sh OUTDIR REPS BATCH "name1:VAR=v VAR2=w" "name2:VAR=u" ...
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; shift; REPS=$1; shift; BATCH=$1; shift
rm -rf $O; mkdir -p $O
for r in $(seq 1 $REPS); do
  for arm in "$@"; do
    name=${arm%%:*}; envs=${arm#*:}
    env $envs timeout -k 10 300 python -u bench.py --batch $BATCH --steps 20 --warmup 5 > $O/${name}_$r.json 2> $O/${name}_$r.err || { tail -20 $O/${name}_$r.err; exit 1; }
    echo "$name rep $r: $(python3 -c "import json,sys; r=json.load(open(sys.argv[1])); print(r['value'], r['ms_per_step'])" $O/${name}_$r.json)"
  done
done
