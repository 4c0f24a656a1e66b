"""BatchNorm kernel bandwidth on ResNet-50 b256 shapes (bn_fwd_from_sums / bn_bwd), HBM GB/s achieved.

    python scripts/bench_bn.py
"""
import json
import os
import sys

sys.path.insert(0, os.environ.get("K8S_AMD_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_amd.ops._ext import load  # noqa: E402

C_ = load()
dev = torch.device("cuda")


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


NB = int(os.environ.get("BN_BATCH", "256"))
SHAPES = [(NB * 112 * 112, 64), (NB * 56 * 56, 64), (NB * 56 * 56, 256), (NB * 28 * 28, 128),
          (NB * 28 * 28, 512), (NB * 14 * 14, 1024), (NB * 7 * 7, 2048)]
for M, C in SHAPES:
    x = torch.randn(M, C, device=dev, dtype=torch.bfloat16)
    res = torch.randn(M, C, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(M, C, device=dev, dtype=torch.bfloat16)
    g = torch.rand(C, device=dev) + 0.5
    b = torch.randn(C, device=dev) * 0.1
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    xf = x.float()
    sums = torch.zeros(C_.conv_stat_replicas, 2, C, device=dev)
    sums[0, 0] = xf.sum(0)
    sums[0, 1] = (xf * xf).sum(0)
    nb = M * C * 2
    out = {"M": M, "C": C}
    for name, r in (("fwd", None), ("fwd_res", res)):
        t = timeit(lambda: C_.bn_fwd_from_sums(x, r, g, b, sums, rm, rv, 0.1, 1e-5, True))
        out[name + "_us"] = round(t * 1e3, 1)
        out[name + "_GBs"] = round(nb * (2 if r is None else 3) / t / 1e6)
    y, mean, invstd = C_.bn_fwd_from_sums(x, res, g, b, sums, rm, rv, 0.1, 1e-5, True)
    dg, db = torch.empty(C, device=dev), torch.empty(C, device=dev)
    t = timeit(lambda: C_.bn_bwd(dy, x, None, mean, invstd, g, b, True, dg, db, False))
    out["bwd_relux_us"] = round(t * 1e3, 1)
    out["bwd_relux_GBs"] = round(nb * 5 / t / 1e6)  # reduce: dy, x; apply: dy, x, dx
    t = timeit(lambda: C_.bn_bwd(dy, x, y, mean, invstd, g, b, False, dg, db, True))
    out["bwd_res_us"] = round(t * 1e3, 1)
    out["bwd_res_GBs"] = round(nb * 8 / t / 1e6)  # reduce: dy, x, y; apply: dy, x, y, dx, dres
    print(json.dumps(out), flush=True)
