"""Time our conv kernels against the vendor path for ResNet-50 b256 shapes, printing any candidate error.

    python scripts/diag_conv.py
"""
import os
import sys
import traceback

os.environ.setdefault("K8S_AMD_AUTOTUNE_CACHE", "none")
sys.path.insert(0, os.environ.get("K8S_AMD_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from k8s_amd.utils.timing import time_ms  # noqa: E402
from k8s_amd.ops import conv  # noqa: E402
from k8s_amd.ops._ext import load  # noqa: E402

C_ = load()
dev = torch.device("cuda")
SHAPES = [  # N, H, C, K, R, stride, pad
    (256, 56, 64, 64, 1, 1, 0),
    (256, 56, 64, 64, 3, 1, 1),
    (256, 56, 64, 256, 1, 1, 0),
    (256, 28, 128, 128, 3, 1, 1),
    (256, 14, 256, 256, 3, 1, 1),
    (256, 7, 512, 2048, 1, 1, 0),
]
for (N, H, C, K, R, s, p) in SHAPES:
    x = torch.randn(N, H, H, C, device=dev, dtype=torch.bfloat16)
    w = torch.randn(K, R, R, C, device=dev, dtype=torch.bfloat16) * 0.05

    def hip():
        st = torch.zeros(C_.conv_stat_replicas, 2, K, device=dev)
        return C_.conv_fwd(x, w, s, p, 1, False, None, 0, st)

    def aten():
        return conv._nhwc(F.conv2d(conv._nchw(x), conv._nchw(w), None, s, p))

    res = {}
    for name, fn in (("hip", hip), ("aten", aten)):
        try:
            res[name] = time_ms(fn, reps=5)
        except Exception as e:  # noqa: BLE001
            res[name] = "ERR " + repr(e)[:300]
            traceback.print_exc()
    try:
        err = (hip().float() - aten().float()).abs().max().item()
    except Exception as e:  # noqa: BLE001
        err = repr(e)[:200]
    flops = 2.0 * N * (H // s) * (H // s) * K * C * R * R
    line = {"shape": (N, H, C, K, R, s, p), "maxerr": err}
    for k, v in res.items():
        line[k + "_ms"] = v
        if isinstance(v, float):
            line[k + "_tflops"] = round(flops / v / 1e9, 1)
    print(line, flush=True)
