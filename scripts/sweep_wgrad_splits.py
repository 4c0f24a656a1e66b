"""Split-K sweep for our weight-gradient kernels on the ResNet-50 b256 shapes: time per split count.

    python scripts/sweep_wgrad_splits.py
"""
import json
import os
import sys

os.environ.setdefault("K8S_AMD_AUTOTUNE_CACHE", "none")
sys.path.insert(0, os.environ.get("K8S_AMD_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_amd.utils.timing import time_ms  # noqa: E402
from k8s_amd.ops._ext import load  # noqa: E402

C_ = load()
dev = torch.device("cuda")
SHAPES = [  # N, H(in), C, K, R, stride, pad
    (256, 14, 256, 256, 3, 1, 1), (256, 14, 512, 512, 3, 2, 1), (256, 28, 256, 256, 3, 2, 1),
    (256, 56, 64, 64, 3, 1, 1), (256, 7, 512, 512, 3, 1, 1), (256, 28, 128, 128, 3, 1, 1),
    (256, 56, 128, 128, 3, 2, 1),
    (256, 56, 256, 128, 1, 1, 0), (256, 56, 256, 64, 1, 1, 0), (256, 56, 64, 256, 1, 1, 0), (256, 56, 64, 64, 1, 1, 0),
    (256, 28, 512, 128, 1, 1, 0), (256, 14, 1024, 256, 1, 1, 0), (256, 7, 2048, 512, 1, 1, 0),
    (256, 7, 512, 2048, 1, 1, 0), (256, 14, 256, 1024, 1, 1, 0),
]
SPLITS = [1, 2, 3, 4, 6, 7, 8, 10, 12, 14, 16, 20, 24, 28, 32, 40, 48, 56, 64, 96, 112, 128, 160, 192, 224, 256, 384, 512, 768, 1024]
for (N, H, C, K, R, s, p) in SHAPES:
    x = torch.randn(N, H, H, C, device=dev, dtype=torch.bfloat16)
    Ho = (H + 2 * p - R) // s + 1
    gy = torch.randn(N, Ho, Ho, K, device=dev, dtype=torch.bfloat16)
    out = torch.empty(K, R, R, C, device=dev, dtype=torch.float32)
    res = {}
    for sp in SPLITS:
        if R == 1 and s == 1:
            fn = lambda: C_.gemm(gy.reshape(-1, K), False, x.reshape(-1, C), False, out.view(K, C), True, None, 0,  # noqa
                                 None, False, 1.0, sp)
        else:
            fn = lambda: C_.conv_wgrad(x, gy, out, s, p, 1, sp, False)  # noqa
        res[sp] = round(time_ms(fn, reps=5) * 1e3, 1)
    if R == 1 and s == 1:
        C_.gemm(gy.reshape(-1, K), False, x.reshape(-1, C), False, out.view(K, C), True, None, 0, None, False, 1.0, 0)
    else:
        C_.conv_wgrad(x, gy, out, s, p, 1, 0, False)
    t_auto = round(time_ms(
        (lambda: C_.gemm(gy.reshape(-1, K), False, x.reshape(-1, C), False, out.view(K, C), True, None, 0, None, False,
                         1.0, 0)) if (R == 1 and s == 1) else (lambda: C_.conv_wgrad(x, gy, out, s, p, 1, 0, False)),
        reps=5) * 1e3, 1)
    best = min(res, key=res.get)
    fl = 2.0 * N * Ho * Ho * K * C * R * R
    print(json.dumps({"shape": [N, H, C, K, R, s, p], "auto_us": t_auto, "best_split": best, "best_us": res[best],
                      "best_tflops": round(fl / res[best] / 1e6), "all": res}), flush=True)
