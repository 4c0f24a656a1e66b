"""Short-K GEMM / 1x1-conv diagnostics: the same product as conv fwd with and without the BN-statistics
epilogue, and as a plain GEMM, for the ResNet-50 shapes the per-layer roofline flags.

    python scripts/conv_ab.py [--batch 1024]
Set PMC_ONLY=<idx> to run just one case 10x (for rocprofv3 --pmc passes).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_amd.ops._ext import load  # noqa: E402

# (name, H, C, K): 1x1 stride-1 convs at batch N -> GEMM M = N*H*H, N = K, K = C
CASES = [("s0.conv3", 56, 64, 256), ("s0.conv1", 56, 256, 64), ("s1.conv3", 28, 128, 512),
         ("s2.conv3", 14, 256, 1024), ("s2.conv1", 14, 1024, 256), ("s0.c1b0", 56, 64, 64)]
# 3x3 stride-1 convs (name, H, C, K): PMC_ONLY=100 + index runs one of these 10x
CASES3 = [("s0.conv2", 56, 64, 64), ("s1.conv2", 28, 128, 128), ("s2.conv2", 14, 256, 256), ("s3.conv2", 7, 512, 512)]


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    a = ap.parse_args()
    C_ = load()
    dev = torch.device("cuda")
    only = os.environ.get("PMC_ONLY")
    if only is not None and int(only) >= 100:
        name, H, C, K = CASES3[int(only) - 100]
        x = torch.randn(a.batch, H, H, C, device=dev, dtype=torch.bfloat16)
        w = (torch.randn(K, 3, 3, C, device=dev) * 0.05).bfloat16()
        st = torch.zeros(C_.conv_stat_replicas, 2, K, device=dev)
        for _ in range(10):
            C_.conv_fwd(x, w, 1, 1, 1, False, None, 0, st)
        torch.cuda.synchronize()
        return
    for i, (name, H, C, K) in enumerate(CASES):
        if only is not None and int(only) != i:
            continue
        x = torch.randn(a.batch, H, H, C, device=dev, dtype=torch.bfloat16)
        w = (torch.randn(K, 1, 1, C, device=dev) * 0.05).bfloat16()
        st = torch.zeros(C_.conv_stat_replicas, 2, K, device=dev)
        M = a.batch * H * H
        fns = {
            "conv_stats": lambda: C_.conv_fwd(x, w, 1, 0, 1, False, None, 0, st),
            "conv": lambda: C_.conv_fwd(x, w, 1, 0, 1, False, None, 0, None),
            "gemm": lambda: C_.gemm(x.view(M, C), True, w.view(K, C), True, None, False, None, 0, None, False, 1.0, 1),
            "blas": lambda: torch.mm(x.view(M, C), w.view(K, C).t()),  # hipBLASLt reference point
            "copy": lambda: torch.empty(M, K, device=dev, dtype=torch.bfloat16).copy_(
                x.view(M, C)[:, :1].expand(M, K)),
        }
        if only is not None:
            for _ in range(10):
                fns["conv_stats"]()
            torch.cuda.synchronize()
            continue
        out = {"case": name, "M": M, "N": K, "K": C}
        nbytes = M * (C + K) * 2
        for k, fn in fns.items():
            t = timed(fn)
            out[k + "_ms"] = round(t, 4)
            out[k + "_tbps"] = round(nbytes / t / 1e9, 2)
        print(json.dumps(out), flush=True)
    if only is None:
        for name, H, C, K in CASES3:
            x = torch.randn(a.batch, H, H, C, device=dev, dtype=torch.bfloat16)
            w = (torch.randn(K, 3, 3, C, device=dev) * 0.05).bfloat16()
            st = torch.zeros(C_.conv_stat_replicas, 2, K, device=dev)
            t = timed(lambda: C_.conv_fwd(x, w, 1, 1, 1, False, None, 0, st))
            flops = 2.0 * a.batch * H * H * K * 9 * C
            print(json.dumps({"case": name + " 3x3", "conv_stats_ms": round(t, 4),
                              "tflops": round(flops / t / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
