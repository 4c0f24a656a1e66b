"""One short-K GEMM shape per process for rocprofv3 --pmc (scripts/gpurun/r4/gsk_pmc.sh): GSK_CASE = fwd (ResNet-50
s1 conv3 forward: 802816 x 128 -> 512, normalize-on-load + statistics) or dgrad (s1 conv1 data gradient: 802816 x
128 -> 512 onto the masked residual gradient). 5 calls."""
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from k8s_amd.ops._ext import load  # noqa: E402

C_ = load()
d = torch.device("cuda")
M, K, N = 802816, 128, 512
case = os.environ.get("GSK_CASE", "fwd")
if case == "fwd":
    x = torch.randn(1, 1, M, K, device=d, dtype=torch.bfloat16)
    w = (torch.randn(N, 1, 1, K, device=d) * K ** -0.5).bfloat16()
    st = torch.zeros(C_.conv_stat_replicas, 2, N, device=d)
    xf = torch.cat([torch.rand(K, device=d) + 0.5, torch.randn(K, device=d) * 0.1]).contiguous()
    f = lambda: C_.conv_fwd(x, w, 1, 0, 1, False, None, 0, st, xform=xf)  # noqa: E731
else:
    gy = torch.randn(M, K, device=d, dtype=torch.bfloat16)
    w = (torch.randn(K, N, device=d) * K ** -0.5).bfloat16()
    dy = torch.randn(M, N, device=d, dtype=torch.bfloat16)
    mask = torch.randint(0, 256, (M * N // 8,), device=d, dtype=torch.uint8)
    out = torch.empty(M, N, device=d, dtype=torch.bfloat16)
    f = lambda: C_.gemm(gy, True, w, False, out, False, None, 0, None, True, 1.0, 1, dy, mask)  # noqa: E731
for _ in range(5):
    f()
torch.cuda.synchronize()
print("ok", case)
