"""BatchNorm per-element pass A/B: forward apply and backward apply at ResNet-50 b1024 shapes, TB/s of compulsory
traffic, under the launch knobs K8S_AMD_BN_UNROLL / K8S_AMD_BN_NT / K8S_AMD_BN_GRID (read once per process, so
every configuration runs in its own child process).

    python scripts/bn_sweep.py                 # sweep
    python scripts/bn_sweep.py --child         # one configuration (environment as given)
"""
import itertools
import json
import os
import subprocess
import sys

SHAPES = [  # (name, M, C, residual)
    ("s0.res", 1024 * 56 * 56, 256, True), ("s0.relu", 1024 * 56 * 56, 64, False),
    ("s2.res", 1024 * 14 * 14, 1024, True), ("s2.relu", 1024 * 14 * 14, 256, False),
]


def child():
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch

    from k8s_amd.ops._ext import load

    C_ = load()
    dev = torch.device("cuda")

    def timed(fn, reps=7):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            fn()
            e.record()
            e.synchronize()
            ts.append(s.elapsed_time(e))
        ts.sort()
        return ts[len(ts) // 2]

    out = {}
    for name, M, C, res in SHAPES:
        x = torch.randn(M, C, device=dev).bfloat16()
        r = torch.randn(M, C, device=dev).bfloat16() if res else None
        g, b = torch.ones(C, device=dev), torch.zeros(C, device=dev)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        sums = torch.zeros(C_.conv_stat_replicas, 2, C, device=dev)
        sums[0, 1] = float(M)
        y, mean, invstd, *mk = C_.bn_fwd_from_sums(x, r, g, b, sums, rm, rv, 0.1, 1e-5, True, res)
        mask = mk[0] if res else None
        t = timed(lambda: C_.bn_fwd_from_sums(x, r, g, b, sums, rm, rv, 0.1, 1e-5, True, res))
        nb = M * C * (4 + (2.125 if res else 0))
        out[name + ".fwd"] = round(nb / t / 1e9, 2)
        dg, db = torch.empty(C, device=dev), torch.empty(C, device=dev)
        t = timed(lambda: C_.bn_bwd(y, x, None, mean, invstd, g, b, not res, dg, db, res, mask))
        nb = M * C * (10 + (2.125 if res else 0))  # reduce reads dy, x; apply reads dy, x, writes dx (+ dres)
        out[name + ".bwd"] = round(nb / t / 1e9, 2)
        del x, r, y
        torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)


def main():
    if "--child" in sys.argv:
        child()
        return
    for u, nt, grid in itertools.product((1, 2), (0, 1), (2048, 4096)):
        env = dict(os.environ, K8S_AMD_BN_UNROLL=str(u), K8S_AMD_BN_NT=str(nt), K8S_AMD_BN_GRID=str(grid))
        r = subprocess.run([sys.executable, __file__, "--child"], env=env, capture_output=True, text=True, timeout=300)
        line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr[-500:]
        print(json.dumps({"unroll": u, "nt": nt, "grid": grid}), line, flush=True)
        if r.returncode != 0:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
