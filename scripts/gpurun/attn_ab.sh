#!/bin/bash
# GPU job: attention tests on this tree, then the attention microbenchmark alternated between this tree (new) and
# abtest/old (the previous kernels) in one session: new, old, new, old.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_attention_gpu.py tests/test_transformer_grads_gpu.py > gpurun_out/attn_test.log 2>&1 || { tail -40 gpurun_out/attn_test.log; exit 1; }
tail -1 gpurun_out/attn_test.log
: > gpurun_out/attn_ab.jsonl
for arm in new old new old; do
  if [ $arm = new ]; then dir=.; else dir=abtest/old; fi
  ( cd $dir && timeout -k 10 200 python -u scripts/bench_attention.py ) > /tmp/attn.jsonl 2> /tmp/attn.err || { tail -5 /tmp/attn.err; exit 1; }
  sed "s/^{/{\"arm\": \"$arm\", /" /tmp/attn.jsonl >> gpurun_out/attn_ab.jsonl
done
python3 - <<'PY'
import json, collections
r = collections.defaultdict(list)
for l in open("gpurun_out/attn_ab.jsonl"):
    d = json.loads(l); r[(d["case"], d["arm"])].append((d["fwd_ms"], d["bwd_ms"]))
for (c, arm), v in sorted(r.items()):
    print(c, arm, "fwd", min(x[0] for x in v), "bwd", min(x[1] for x in v))
PY
