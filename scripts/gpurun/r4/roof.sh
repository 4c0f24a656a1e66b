#!/bin/bash
# GPU job (round 4): per-layer ResNet-50 b1024 roofline with speed-of-light floors.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u scripts/layer_roofline.py --reps 5 > gpurun_out/r4_roof2.jsonl 2> gpurun_out/r4_roof.err || { tail -30 gpurun_out/r4_roof.err; exit 1; }
python3 - <<'PY'
import json
rows = [json.loads(l) for l in open("gpurun_out/r4_roof2.jsonl")]
print(rows[-1])
for r in sorted(rows[:-1], key=lambda r: -r.get("lost_ms_per_step", 0))[:30]:
    print("%-12s %-6s x%d %7.3f ms  step %6.3f  sol %.2f  lost %6.3f" % (r["layer"], r["op"], r["count"], r["ms"], r["step_ms"], r["sol"], r["lost_ms_per_step"]))
PY
