"""Debug: attention_qkv rope in place vs copy (which rows / heads differ, and is the copy form deterministic)."""
import torch

from k8s_amd.ops import nn as K
from k8s_amd.ops.attention import attention_qkv

torch.manual_seed(9)
B, S, H, Hkv, D = 2, 256, 8, 2, 128
W = (H + 2 * Hkv) * D
dev = torch.device("cuda")
base = (torch.randn(B * S, W, device=dev) * 0.5).bfloat16()
pos = torch.arange(S, device=dev, dtype=torch.int32).repeat(B)
table = K.rope_table(S, D, device=dev)
res = {}
for name, ip in (("copy", False), ("copy2", False), ("inplace", True)):
    qkv = base.clone()
    with torch.no_grad():
        o = attention_qkv(qkv, B, S, H, Hkv, D, causal=True, rope=(pos, table), rope_in_place=ip)
    res[name] = (o.float(), qkv.float())
    print(name, "qkv changed:", (qkv.float() - base.float()).abs().max().item())
for a, b in (("copy", "copy2"), ("copy", "inplace")):
    d = (res[a][0] - res[b][0]).abs()
    print(a, b, "max diff", d.max().item(), "rows", (d.amax(dim=(2, 3)) > 0).nonzero()[:5].tolist())
