"""rocprofv3 --pmc driver for the flash-attention kernels at Llama-3-8B shape (s4096, 32 / 8 heads, D 128, causal):
5 forward + 5 backward launches.

    rocprofv3 --pmc SQ_WAVES ... -d gpurun_out/pmc_attn -o p -- python scripts/pmc_attention.py
"""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_amd.ops._ext import load  # noqa: E402

C = load()
dev = torch.device("cuda")
torch.manual_seed(0)
# ATTN_SHAPE=bert: BERT-base s128 b1024 (12 heads, D 64, non-causal) instead
if os.environ.get("ATTN_SHAPE") == "bert":
    B, S, Hq, Hkv, D, causal = 1024, 128, 12, 12, 64, False
else:
    B, S, Hq, Hkv, D, causal = 1, 4096, 32, 8, 128, True
q = torch.randn(B, S, Hq, D, device=dev).bfloat16()
k = torch.randn(B, S, Hkv, D, device=dev).bfloat16()
v = torch.randn(B, S, Hkv, D, device=dev).bfloat16()
sc = 1.0 / math.sqrt(D)
o, lse = C.flash_fwd(q, k, v, causal, None, sc)
do = torch.randn_like(o)
for _ in range(5):
    C.flash_fwd(q, k, v, causal, None, sc)
    C.flash_bwd(do, q, k, v, o, lse, causal, None, sc)
torch.cuda.synchronize()
print("ok")
