"""Small driver for rocprofv3 --pmc passes: a few hot k8s_amd kernels, 10 launches each.

    rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES ... -d gpurun_out/pmc -o run -- python scripts/pmc_kernels.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_amd.ops._ext import load  # noqa: E402

C = load()
dev = torch.device("cuda")
torch.manual_seed(0)
x3 = torch.randn(256, 14, 14, 256, device=dev).bfloat16()
w3 = (torch.randn(256, 3, 3, 256, device=dev) * 0.05).bfloat16()
a = torch.randn(8192, 768, device=dev).bfloat16()
b = torch.randn(2304, 768, device=dev).bfloat16()
g1 = torch.randn(256 * 56 * 56, 256, device=dev).bfloat16()
w1 = torch.randn(256, 64, device=dev).bfloat16()
for _ in range(10):
    C.conv_fwd(x3, w3, 1, 1, 1, False, None, 0, None)                            # 3x3 implicit GEMM
    C.gemm(a, True, b, True, None, False, None, 0, None, False, 1.0, 1)           # BERT QKV
    C.gemm(g1, True, w1, False, None, False, None, 0, None, False, 1.0, 1)        # 1x1 dgrad (w read N-major)
torch.cuda.synchronize()
print("ok")
