"""Drive one product shape in one form through our GEMM and through torch.mm (hipBLASLt), a few reps each, for
rocprofv3 kernel-trace / PMC passes: the vendor kernel's name (its macro tile / depth / prefetch settings) and its
counters next to ours on the same operands.

    BV_SHAPE=4096,28672,4096 BV_FORM=fwd python scripts/blas_vs_ours.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from k8s_amd.ops._ext import load  # noqa: E402

C = load()
d = torch.device("cuda")
M, N, K = (int(v) for v in os.environ.get("BV_SHAPE", "4096,28672,4096").split(","))
form = os.environ.get("BV_FORM", "fwd")
reps = int(os.environ.get("BV_REPS", "5"))
x = (torch.rand(M, K, device=d) * 2 - 1).bfloat16()
w = (torch.rand(N, K, device=d) * 2 - 1).bfloat16()
g = (torch.rand(M, N, device=d) * 2 - 1).bfloat16()
dw = torch.empty(N, K, device=d)
if form == "fwd":
    ours, blas = (lambda: C.gemm(x, True, w, True, None, False, None, 0, None, False, 1.0, 1)), (lambda: x @ w.t())
elif form == "dgrad":
    ours, blas = (lambda: C.gemm(g, True, w, False, None, False, None, 0, None, False, 1.0, 1)), (lambda: g @ w)
else:
    ours, blas = (lambda: C.gemm(g, False, x, False, dw, True, None, 0, None, False, 1.0, 0)), (lambda: g.t() @ x)
who = os.environ.get("BV_WHO", "both")
for _ in range(reps):
    if who in ("both", "ours"):
        ours()
    if who in ("both", "blas"):
        blas()
torch.cuda.synchronize()
print("done")
