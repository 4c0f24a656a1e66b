"""Drive the staged-window 3x3 conv on the ResNet-50 b1024 stride-1 shapes for rocprofv3 --pmc passes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from k8s_amd.ops._ext import load  # noqa: E402

C_ = load()
dev = torch.device("cuda")
for H, C, K in [(56, 64, 64), (28, 128, 128), (14, 256, 256)]:
    x = (torch.rand(1024, H, H, C, device=dev) * 2 - 1).bfloat16()
    w = ((torch.rand(K, 3, 3, C, device=dev) * 2 - 1) / (3 * C ** 0.5)).bfloat16()
    st = torch.zeros(C_.conv_stat_replicas, 2, K, device=dev)
    for _ in range(3):
        C_.conv_fwd(x, w, 1, 1, 1, False, None, 0, st)
torch.cuda.synchronize()
print("done")
