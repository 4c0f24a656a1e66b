#!/usr/bin/env python3
"""Stem max-pool microbenchmark (ResNet-50 b1024: [1024, 112, 112, 64] bf16, 3x3 / s2 / p1): forward and backward
time and effective HBM bandwidth (compulsory bytes: x + y + idx forward, dy + idx + dx backward). One JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_amd.ops._ext import load  # noqa: E402


def bench(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / it * 1e-3


def main():
    C = load()
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    x = torch.randn(N, 112, 112, 64, device="cuda").bfloat16()
    y, idx = C.maxpool_fwd(x, 3, 2, 1)
    dy = torch.randn_like(y)
    tf = bench(lambda: C.maxpool_fwd(x, 3, 2, 1))
    tb = bench(lambda: C.maxpool_bwd(dy, idx, 112, 112, 3, 2, 1))
    bf = x.numel() * 2 + y.numel() * 2 + idx.numel()
    bb = dy.numel() * 2 + idx.numel() + x.numel() * 2
    print(json.dumps({"N": N, "fwd_us": round(tf * 1e6, 1), "fwd_TBps": round(bf / tf / 1e12, 2),
                      "bwd_us": round(tb * 1e6, 1), "bwd_TBps": round(bb / tb / 1e12, 2)}), flush=True)


if __name__ == "__main__":
    main()
