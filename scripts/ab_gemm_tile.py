"""A/B of the GEMM main loop: 128x128 tiles with two LDS buffers (K8S_AMD_GEMM_PIPE=0) vs 256x128 tiles, 8 waves,
and ResNet-50 convolutions, same process, interleaved; also checks the 256x128 results against 128x128.

    python scripts/ab_gemm_tile.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_amd.utils.timing import time_ms  # noqa: E402
from k8s_amd.ops._ext import load  # noqa: E402

C = load()
dev = torch.device("cuda")


def t(fn):
    return time_ms(fn, reps=7)


GEMMS = [("bert_qkv", 8192, 2304, 768), ("bert_ffn1", 8192, 3072, 768), ("bert_ffn2", 8192, 768, 3072),
         ("bert_out", 8192, 768, 768), ("llama1b_qkv", 4096, 3072, 2048), ("llama_down", 4096, 4096, 14336),
         ("sq8192", 8192, 8192, 8192), ("rn_1x1_56", 802816, 256, 64), ("rn_1x1_14", 50176, 1024, 256)]
for name, M, N, K in GEMMS:
    a = torch.randn(M, K, device=dev).bfloat16()
    b = torch.randn(N, K, device=dev).bfloat16()
    res = {}
    outs = {}
    for tile in ("1", "2", "1", "2"):
        os.environ["K8S_AMD_GEMM_PIPE"] = {"1": "0", "2": "1"}[tile]
        fn = lambda: C.gemm(a, True, b, True, None, False, None, 0, None, False, 1.0, 1)  # noqa: E731
        res.setdefault(tile, []).append(t(fn))
        outs[tile] = fn()
    err = ((outs["1"].float() - outs["2"].float()).norm() / outs["1"].float().norm()).item()
    r = {k: min(v) for k, v in res.items()}
    fl = 2.0 * M * N * K
    print(json.dumps({"gemm": name, "MNK": [M, N, K], "t2buf_us": round(r["1"] * 1e3, 1), "t3stage_us": round(r["2"] * 1e3, 1),
                      "tf2buf": round(fl / r["1"] / 1e9), "tf3stage": round(fl / r["2"] / 1e9), "relerr": err}), flush=True)
CONVS = [(256, 56, 64, 64, 3, 1, 1), (256, 28, 128, 128, 3, 1, 1), (256, 14, 256, 256, 3, 1, 1),
         (256, 7, 512, 512, 3, 1, 1), (256, 56, 64, 256, 1, 1, 0), (256, 56, 256, 64, 1, 1, 0),
         (256, 28, 512, 128, 1, 1, 0), (256, 14, 256, 1024, 1, 1, 0), (256, 56, 128, 128, 3, 2, 1)]
for (N, H, Cin, K, R, s, p) in CONVS:
    x = torch.randn(N, H, H, Cin, device=dev).bfloat16()
    w = (torch.randn(K, R, R, Cin, device=dev) * 0.05).bfloat16()
    res, outs = {}, {}
    for tile in ("1", "2", "1", "2"):
        os.environ["K8S_AMD_GEMM_PIPE"] = {"1": "0", "2": "1"}[tile]
        fn = lambda: C.conv_fwd(x, w, s, p, 1, False, None, 0, None)  # noqa: E731
        res.setdefault(tile, []).append(t(fn))
        outs[tile] = fn()
    err = ((outs["1"].float() - outs["2"].float()).norm() / outs["1"].float().norm()).item()
    r = {k: min(v) for k, v in res.items()}
    Ho = (H + 2 * p - R) // s + 1
    fl = 2.0 * N * Ho * Ho * K * Cin * R * R
    print(json.dumps({"conv": [N, H, Cin, K, R, s, p], "t2buf_us": round(r["1"] * 1e3, 1), "t3stage_us": round(r["2"] * 1e3, 1),
                      "tf2buf": round(fl / r["1"] / 1e9), "tf3stage": round(fl / r["2"] / 1e9), "relerr": err}), flush=True)
os.environ.pop("K8S_AMD_GEMM_PIPE", None)
