"""HBM bandwidth reference points on this GPU: read-only, write-only and copy of a large bf16 buffer (PyTorch's
own kernels), so per-kernel TB/s figures in profiles/ have a measured ceiling next to them.

    python scripts/membw.py [--gb 2]
"""
import argparse
import json

import torch


def timed(fn, reps=10):
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=2.0)
    a = ap.parse_args()
    n = int(a.gb * 2**30 / 2)
    x = torch.randn(n, device="cuda").bfloat16()
    y = torch.empty_like(x)
    out = {"bytes": 2 * n}
    t = timed(lambda: x.sum())
    out["read_tbps"] = round(2 * n / t / 1e9, 2)
    t = timed(lambda: y.fill_(1.0))
    out["write_tbps"] = round(2 * n / t / 1e9, 2)
    t = timed(lambda: y.copy_(x))
    out["copy_tbps"] = round(4 * n / t / 1e9, 2)
    t = timed(lambda: torch.add(x, x, out=y))
    out["add_tbps"] = round(4 * n / t / 1e9, 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
