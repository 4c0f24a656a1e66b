#!/bin/bash
# GPU job: headline bench A/B between this tree (new) and abtest/old (a copy with the previous kernels), alternated
# in one session on one box: new, old, new, old.
set -o pipefail
mkdir -p gpurun_out
for arm in new old new old; do
  if [ $arm = new ]; then dir=.; else dir=abtest/old; fi
  ( cd $dir && timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 2> /tmp/ab.err ) > /tmp/ab.json || { tail -5 /tmp/ab.err; exit 1; }
  echo "$arm $(python3 -c "import json;d=json.load(open('/tmp/ab.json'));print(d['value'], d['ms_per_step'])")"
done
