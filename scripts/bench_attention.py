#!/usr/bin/env python3
"""Flash-attention microbenchmark: our gfx950 kernels vs torch SDPA on the BERT / Llama shapes.
One JSON line per case (TFLOP/s counted as 4*B*H*S*S*D fwd (x0.5 causal), 2.5x that for bwd)."""
import json
import math
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_amd.ops._ext import load  # noqa: E402


def bench(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / it * 1e-3


def main():
    C = load()
    cases = [("bert_s128", 64, 128, 12, 12, 64, False), ("bert_s128_b1024", 1024, 128, 12, 12, 64, False), ("bert_s512", 16, 512, 12, 12, 64, False),
             ("llama_s2048", 2, 2048, 32, 8, 128, True), ("llama1b_s2048_d64", 2, 2048, 32, 8, 64, True), ("llama_s4096", 1, 4096, 32, 8, 128, True),
             ("mha_s4096_nc", 1, 4096, 32, 32, 128, False)]
    only = os.environ.get("ATTN_CASES")
    for name, B, S, Hq, Hkv, D, causal in cases:
        if only and name not in only.split(","):
            continue
        q = torch.randn(B, S, Hq, D, device="cuda").bfloat16()
        k = torch.randn(B, S, Hkv, D, device="cuda").bfloat16()
        v = torch.randn(B, S, Hkv, D, device="cuda").bfloat16()
        sc = 1.0 / math.sqrt(D)
        flops = 4.0 * B * Hq * S * S * D * (0.5 if causal else 1.0)
        o, lse = C.flash_fwd(q, k, v, causal, None, sc)
        do = torch.randn_like(o)
        tf = bench(lambda: C.flash_fwd(q, k, v, causal, None, sc))
        tb = bench(lambda: C.flash_bwd(do, q, k, v, o, lse, causal, None, sc))
        rec = {"case": name, "B": B, "S": S, "Hq": Hq, "Hkv": Hkv, "D": D, "causal": causal,
               "fwd_ms": round(tf * 1e3, 3), "fwd_tflops": round(flops / tf / 1e12, 1),
               "bwd_ms": round(tb * 1e3, 3), "bwd_tflops": round(2.5 * flops / tb / 1e12, 1)}
        try:
            qt, kt, vt = (t.transpose(1, 2) for t in (q, k, v))
            if Hkv != Hq:
                kt = kt.repeat_interleave(Hq // Hkv, 1)
                vt = vt.repeat_interleave(Hq // Hkv, 1)
            sd = torch.nn.functional.scaled_dot_product_attention
            t2 = bench(lambda: sd(qt, kt, vt, is_causal=causal))
            rec["sdpa_fwd_ms"] = round(t2 * 1e3, 3)
            rec["sdpa_fwd_tflops"] = round(flops / t2 / 1e12, 1)
        except Exception as e:  # noqa: BLE001
            rec["sdpa_error"] = str(e)[:100]
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
