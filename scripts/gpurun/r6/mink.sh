#!/bin/bash
# GPU job (round 6): per-layer fwd / dgrad / wgrad timings with and without K = 512 on the 4-wave GEMM.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_mink; rm -rf $O; mkdir -p $O
for m in 768 512; do
  K8S_AMD_GEMM256_MINK=$m timeout -k 10 300 python -u scripts/layer_roofline.py --batch 3072 --reps 5 --only fwd,dgrad,wgrad > $O/roof_$m.jsonl 2> $O/roof_$m.err || { tail -20 $O/roof_$m.err; exit 1; }
done
python3 - <<'PY'
import json
a={(r['layer'],r['op']):r['ms'] for r in map(json.loads,open('gpurun_out/r6_mink/roof_768.jsonl')) if 'layer' in r}
b={(r['layer'],r['op']):r['ms'] for r in map(json.loads,open('gpurun_out/r6_mink/roof_512.jsonl')) if 'layer' in r}
for k in a:
    if abs(a[k]-b[k])/a[k] > 0.03: print(k, a[k], b[k])
PY
