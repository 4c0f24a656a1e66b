"""ResNet-50 weight gradients at batch 1024 on the shapes MIOpen took in round 1: our streaming kernel
(wgrad_stream.hip), our generic split-K GEMM (K8S_AMD_WGRAD_STREAM=0) and MIOpen, interleaved in one process.

    python scripts/bench_wgrad.py [--batch 1024]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from k8s_amd.ops import conv  # noqa: E402
from k8s_amd.ops._ext import load  # noqa: E402

C_ = load()
dev = torch.device("cuda")
SHAPES = [  # H(in), C, K, R, stride, pad
    (56, 64, 64, 1, 1, 0), (56, 64, 256, 1, 1, 0), (56, 256, 64, 1, 1, 0), (56, 256, 128, 1, 1, 0),
    (56, 256, 512, 1, 2, 0), (28, 128, 512, 1, 1, 0), (28, 512, 128, 1, 1, 0), (28, 512, 256, 1, 1, 0),
    (56, 128, 128, 3, 2, 1), (28, 256, 256, 3, 2, 1), (14, 512, 512, 3, 2, 1),
]


def t(fn, reps=5):
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
    ap.add_argument("--batch", type=int, default=1024)
    a = ap.parse_args()
    N = a.batch
    for (H, C, K, R, s, p) in SHAPES:
        x = torch.randn(N, H, H, C, device=dev).bfloat16()
        w = (torch.randn(K, R, R, C, device=dev) * 0.05).bfloat16()
        Ho = (H + 2 * p - R) // s + 1
        gy = torch.randn(N, Ho, Ho, K, device=dev).bfloat16()
        dw = torch.empty(K, R, R, C, device=dev)
        elig = C_.wgrad_stream_eligible(N, Ho, Ho, C, K, R, R)
        res = {"stream": [], "generic": [], "miopen": []}
        for _ in range(3):
            os.environ.pop("K8S_AMD_WGRAD_STREAM", None)
            res["stream"].append(t(lambda: C_.conv_wgrad(x, gy, dw, s, p, 1, 0, False)))
            os.environ["K8S_AMD_WGRAD_STREAM"] = "0"
            res["generic"].append(t(lambda: C_.conv_wgrad(x, gy, dw, s, p, 1, 0, False)))
            os.environ.pop("K8S_AMD_WGRAD_STREAM", None)
            res["miopen"].append(t(lambda: conv._aten_bwd(gy, x, w, s, p, False, True)))
        C_.conv_wgrad(x, gy, dw, s, p, 1, 0, False)
        ref = conv._aten_bwd(gy, x, w, s, p, False, True)[1].float()
        err = ((dw - ref).norm() / ref.norm()).item()
        byts = 2 * (x.numel() + gy.numel())
        best = {k: min(v) for k, v in res.items()}
        print(json.dumps({"shape": [N, H, C, K, R, s, p], "eligible": elig,
                          **{k + "_us": round(v, 1) for k, v in best.items()},
                          "stream_GBs": round(byts / best["stream"] / 1e3), "relerr_vs_miopen": round(err, 5)}),
              flush=True)
        del x, w, gy, dw
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
