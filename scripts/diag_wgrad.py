"""Our conv backward (wgrad / dgrad) vs the vendor path on the ResNet-50 b256 shapes where MIOpen won the
autotune (profiles/: conv_wgrad 3x3 + 1x1@56x56, strided dgrad).

    python scripts/diag_wgrad.py
"""
import json
import os
import sys

os.environ.setdefault("K8S_AMD_AUTOTUNE_CACHE", "none")
sys.path.insert(0, os.environ.get("K8S_AMD_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_amd.ops import conv  # noqa: E402
from k8s_amd.utils.timing import time_ms  # noqa: E402
from k8s_amd.ops._ext import load  # noqa: E402

C_ = load()
dev = torch.device("cuda")
WGRAD = [  # N, H(in), C, K, R, stride, pad
    (256, 14, 256, 256, 3, 1, 1), (256, 14, 512, 512, 3, 2, 1), (256, 28, 256, 256, 3, 2, 1),
    (256, 56, 256, 128, 1, 1, 0), (256, 56, 256, 64, 1, 1, 0), (256, 56, 64, 256, 1, 1, 0),
    (256, 56, 64, 64, 1, 1, 0), (256, 56, 64, 64, 3, 1, 1), (256, 7, 512, 512, 3, 1, 1),
    (256, 28, 128, 128, 3, 1, 1), (256, 56, 128, 128, 3, 2, 1),
]
for (N, H, C, K, R, s, p) in WGRAD:
    x = torch.randn(N, H, H, C, device=dev, dtype=torch.bfloat16)
    w = torch.randn(K, R, R, C, device=dev, dtype=torch.bfloat16) * 0.05
    Ho = (H + 2 * p - R) // s + 1
    gy = torch.randn(N, Ho, Ho, K, device=dev, dtype=torch.bfloat16)
    out = torch.empty(K, R, R, C, device=dev, dtype=torch.float32)
    t_hip = time_ms(lambda: conv._wgrad_hip(C_, gy, x, out, s, p, False), reps=5)
    t_aten = time_ms(lambda: conv._aten_bwd(gy, x, w, s, p, False, True), reps=5)
    conv._wgrad_hip(C_, gy, x, out, s, p, False)
    ref = conv._aten_bwd(gy, x, w, s, p, False, True)[1].float()
    err = ((out - ref).abs().max() / ref.abs().max()).item()
    fl = 2.0 * N * Ho * Ho * K * C * R * R
    byts = 2 * (x.numel() + gy.numel())
    print(json.dumps({"op": "wgrad", "shape": [N, H, C, K, R, s, p], "hip_us": round(t_hip * 1e3, 1),
                      "aten_us": round(t_aten * 1e3, 1), "hip_tflops": round(fl / t_hip / 1e9),
                      "hip_GBs": round(byts / t_hip / 1e6), "relerr": round(err, 5)}), flush=True)
DGRAD_S2 = [(256, 56, 128, 128, 3, 2, 1), (256, 28, 256, 256, 3, 2, 1), (256, 14, 512, 512, 3, 2, 1),
            (256, 56, 256, 512, 1, 2, 0), (256, 28, 512, 1024, 1, 2, 0), (256, 14, 1024, 2048, 1, 2, 0)]
for (N, H, C, K, R, s, p) in DGRAD_S2:
    x = torch.randn(N, H, H, C, device=dev, dtype=torch.bfloat16)
    w = torch.randn(K, R, R, C, device=dev, dtype=torch.bfloat16) * 0.05
    Ho = (H + 2 * p - R) // s + 1
    gy = torch.randn(N, Ho, Ho, K, device=dev, dtype=torch.bfloat16)
    t_aten = time_ms(lambda: conv._aten_bwd(gy, x, w, s, p, True, False), reps=5)
    t_hip = time_ms(lambda: conv._dgrad_strided_hip(C_, gy, w, s, p, H, H), reps=5)
    ref = conv._aten_bwd(gy, x, w, s, p, True, False)[0].float()
    err = ((conv._dgrad_strided_hip(C_, gy, w, s, p, H, H).float() - ref).norm() / ref.norm()).item()
    fl = 2.0 * N * Ho * Ho * K * C * R * R
    print(json.dumps({"op": "dgrad_s2", "shape": [N, H, C, K, R, s, p], "aten_us": round(t_aten * 1e3, 1),
                      "hip_us": round(t_hip * 1e3, 1), "aten_tflops": round(fl / t_aten / 1e9),
                      "hip_tflops": round(fl / t_hip / 1e9), "relerr": round(err, 5)}), flush=True)
