"""ResNet-50 1x1 convolutions as plain GEMMs on the 128 x 128 kernel (gemm.hip) vs the 256 x 256 LDS-ring kernel
(gemm256.hip), forward / data gradient / weight gradient, at the bench batch.

    python scripts/gemm_1x1_ab.py [--batch 1024]

One JSON line per (layer, op): ms of each kernel and the ratio; K8S_AMD_GEMM256 is switched per call (0 = 128
kernel, 2 = 256 kernel wherever it can take the shape).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_amd.ops._ext import load  # noqa: E402


def layers():
    out, cin, H = [], 64, 56
    for si, (nb, w) in enumerate([(3, 64), (4, 128), (6, 256), (3, 512)]):
        s = 1 if si == 0 else 2
        Ho = H // s
        out.append(("s%d.b0.conv1" % si, H, cin, w))
        out.append(("s%d.b0.conv3" % si, Ho, w, 4 * w))
        out.append(("s%d.bx.conv1" % si, Ho, 4 * w, w))
        cin, H = 4 * w, Ho
    return out


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
    for name, H, C, K in layers():
        M = a.batch * H * H
        x = torch.randn(M, C, device=dev, dtype=torch.bfloat16)
        dy = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = (torch.randn(K, C, device=dev) * 0.05).bfloat16()
        dw = torch.empty(K, C, device=dev, dtype=torch.float32)
        ops = {
            "fwd": lambda: C_.gemm(x, True, w, True, None, False, None, 0, None, False, 1.0, 1),
            "dgrad": lambda: C_.gemm(dy, True, w, False, None, False, None, 0, None, False, 1.0, 1),
            "wgrad": lambda: C_.gemm(dy, False, x, False, dw, True, None, 0, None, False, 1.0, 0),
        }
        for op, fn in ops.items():
            r = {"layer": name, "op": op, "M": M, "C": C, "K": K}
            for mode in ("0", "2"):
                os.environ["K8S_AMD_GEMM256"] = mode
                r["ms_" + ("g128" if mode == "0" else "g256")] = round(timed(fn), 4)
            r["g256_speedup"] = round(r["ms_g128"] / r["ms_g256"], 3)
            print(json.dumps(r), flush=True)
        del x, dy, w, dw
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
