"""Drive the 256 x 256 GEMM on one shape per operand layout, for rocprofv3 --pmc passes (scripts/gpurun/pmc_gemm256.sh)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from k8s_amd.ops._ext import load  # noqa: E402

C = load()
d = torch.device("cuda")
M = N = K = int(os.environ.get("PMC_MNK", "4096"))
x = (torch.rand(M, K, device=d) * 2 - 1).bfloat16()
w = (torch.rand(N, K, device=d) * 2 - 1).bfloat16()
g = (torch.rand(M, N, device=d) * 2 - 1).bfloat16()
for _ in range(int(os.environ.get("PMC_REPS", "10"))):
    C.gemm(x, True, w, True, None, False, None, 0, None, False, 1.0, 1)
    C.gemm(g, True, w, False, None, False, None, 0, None, False, 1.0, 1)
torch.cuda.synchronize()
print("done")
