"""Stem A/B: the 7x7 / stride-2 conv over the 8-channel-padded image vs the equivalent 4x4 / stride-1 conv over
its 2x2 space-to-depth transform (16 channels), forward (with BN statistics) and weight gradient, batch 1024."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from k8s_amd.ops import conv  # noqa: E402
from k8s_amd.ops._ext import load  # noqa: E402


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


C_ = load()
dev = torch.device("cuda")
N = int(os.environ.get("BATCH", "1024"))
for name, H, C, R, st, pad in (("7x7s2_c8", 224, 8, 7, 2, 3), ("4x4s1_c16_s2d", 115, 16, 4, 1, 0)):
    x = torch.randn(N, H, H, C, device=dev).bfloat16()
    w = (torch.randn(64, R, R, C, device=dev) * 0.05).bfloat16()
    Ho = (H + 2 * pad - R) // st + 1
    gy = torch.randn(N, Ho, Ho, 64, device=dev).bfloat16()
    stt = torch.zeros(C_.conv_stat_replicas, 2, 64, device=dev)
    dw = torch.empty(64, R, R, C, device=dev)
    tf = timed(lambda: C_.conv_fwd(x, w, st, pad, 1, False, None, 0, stt))
    tw = timed(lambda: conv._wgrad_hip(C_, gy, x, dw, st, pad, False))
    print(json.dumps({"stem": name, "Ho": Ho, "fwd_ms": round(tf, 3), "wgrad_ms": round(tw, 3)}), flush=True)
