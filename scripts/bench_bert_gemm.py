#!/usr/bin/env python3
"""BERT-base b1024 (M = 131072 tokens) linear products at training size, with the trainer's epilogues: forward with
bias (FFN1: + GELU and the pre-activation copy), plain data gradients. One JSON line per product (us, TF/s); A/B
knobs are environment variables read once per process (e.g. K8S_AMD_G4_STAGGER), so compare separate runs.

    python scripts/bench_bert_gemm.py [--reps 10]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_amd.ops._ext import load  # noqa: E402


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--M", type=int, default=131072)
    ap.add_argument("--blas", action="store_true", help="also plain forwards and hipBLASLt (torch.mm) arms")
    a = ap.parse_args()
    C = load()
    dev = torch.device("cuda")
    M = a.M
    rnd = lambda *s: (torch.rand(*s, device=dev) * 2 - 1).bfloat16()  # noqa: E731
    for name, N, K, act in [("qkv", 2304, 768, 0), ("o", 768, 768, 0), ("ffn1", 3072, 768, 2), ("ffn2", 768, 3072, 0)]:
        x, w, g = rnd(M, K), rnd(N, K), rnd(M, N)
        b = torch.randn(N, device=dev)
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        pre = torch.empty_like(y) if act else None
        dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
        fwd = lambda: C.gemm(x, True, w, True, y, False, b, act, pre, False, 1.0, 1)  # noqa: E731
        dgr = lambda: C.gemm(g, True, w, False, dx, False, None, 0, None, False, 1.0, 1)  # noqa: E731
        cases = [("fwd", fwd), ("dgrad", dgr)]
        if a.blas:  # the same products without epilogue extras, ours vs hipBLASLt (torch.mm)
            cases += [("fwd_plain", lambda: C.gemm(x, True, w, True, y, False, None, 0, None, False, 1.0, 1)),
                      ("fwd_plain_blas", lambda: torch.mm(x, w.t(), out=y)),
                      ("dgrad_blas", lambda: torch.mm(g, w, out=dx))]
        for form, fn in cases:
            us = min(timeit(fn, a.reps) for _ in range(3))
            print(json.dumps({"layer": name, "form": form, "MNK": [M, K, N] if form.startswith("dgrad") else [M, N, K],
                              "us": round(us, 1), "tf": round(2.0 * M * N * K / us / 1e6),
                              "stagger": os.environ.get("K8S_AMD_G4_STAGGER", "0")}), flush=True)
        del x, w, g, y, pre, dx


if __name__ == "__main__":
    main()
