#!/bin/bash
# GPU job (round 5): weight gradients on a side stream (K8S_AMD_WGRAD_STREAM) -- numerics test, then the headline
# bench A/B/A/B on one box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_wside; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_resnet_gpu.py -k "side_stream or gradients_match" > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -3 $O/test.log
for arm in 0 1 0 1; do
  K8S_AMD_WGRAD_STREAM=$arm timeout -k 10 300 python -u bench.py --steps ${STEPS:-20} --warmup 5 ${BATCH:+--batch $BATCH} > $O/b$arm.json 2> $O/b$arm.err || { tail -20 $O/b$arm.err; exit 1; }
  echo "arm $arm: $(python -c "import json,sys; d=json.load(open('$O/b$arm.json')); print(d['value'], d['ms_per_step'], d['peak_mem_gb'])")"
  cat $O/b$arm.json >> $O/ab.jsonl
done
