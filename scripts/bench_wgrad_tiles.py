"""Weight-gradient tile A/B (csrc/kernels/wgrad_stream.hip, $K8S_AMD_WGS_TILE) on every ResNet-50 weight-gradient
shape at the bench batch, with the generic split-K kernel as the other reference point; prints TFLOP/s and the
relative difference of each variant to the generic kernel's result.

    python scripts/bench_wgrad_tiles.py [--batch 1024]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from k8s_amd.ops._ext import load  # noqa: E402

SHAPES = [  # H(in), C, K, R, stride, pad
    (56, 64, 64, 3, 1, 1), (28, 128, 128, 3, 1, 1), (14, 256, 256, 3, 1, 1), (7, 512, 512, 3, 1, 1),
    (56, 128, 128, 3, 2, 1), (28, 256, 256, 3, 2, 1), (14, 512, 512, 3, 2, 1),
    (56, 64, 256, 1, 1, 0), (56, 256, 64, 1, 1, 0), (28, 128, 512, 1, 1, 0), (28, 512, 128, 1, 1, 0),
    (14, 256, 1024, 1, 1, 0), (14, 1024, 256, 1, 1, 0), (7, 512, 2048, 1, 1, 0), (7, 2048, 512, 1, 1, 0),
    (56, 256, 128, 1, 1, 0), (56, 256, 512, 1, 2, 0), (28, 512, 256, 1, 1, 0), (28, 512, 1024, 1, 2, 0),
    (14, 1024, 512, 1, 1, 0), (14, 1024, 2048, 1, 2, 0),
]
TILES = [t for t in os.environ.get("WGS_TILES", "128x64,128x128,256x128,64x64").split(",") if "x" in t]


def timed(fn, reps=5):
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
    N = a.batch
    for (H, C, K, R, s, p) in SHAPES:
        torch.manual_seed(0)
        x = torch.randn(N, H, H, C, device=dev).bfloat16()
        Ho = (H + 2 * p - R) // s + 1
        gy = torch.randn(N, Ho, Ho, K, device=dev).bfloat16()
        dw = torch.empty(K, R, R, C, device=dev)
        flops = 2.0 * N * Ho * Ho * K * R * R * C
        out = {"shape": [N, H, C, K, R, s, p]}
        out["generic_tf"] = round(flops / timed(lambda: C_.conv_wgrad(x, gy, dw, s, p, 1, 0, False)) / 1e9, 1)
        ref = dw.clone()
        os.environ["K8S_AMD_WGS_ANY"] = "1"  # time the streaming kernel on every shape
        for tile in TILES:
            os.environ["K8S_AMD_WGS_TILE"] = tile
            kt, ct = map(int, tile.split("x"))
            if K % kt or (R * R * C) % ct or not C_.wgrad_stream_eligible(N, Ho, Ho, C, K, R, R):
                continue
            ms = timed(lambda: C_.conv_wgrad(x, gy, dw, s, p, 1, 0, False))
            out[tile + "_tf"] = round(flops / ms / 1e9, 1)
            out[tile + "_err"] = float("%.2e" % ((dw - ref).norm() / ref.norm()).item())
        os.environ.pop("K8S_AMD_WGS_TILE", None)
        os.environ.pop("K8S_AMD_WGS_ANY", None)
        print(json.dumps(out), flush=True)
        del x, gy, dw, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
