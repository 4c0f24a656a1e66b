#!/usr/bin/env python3
"""Kernel microbenchmarks on one MI355X: our MFMA GEMM / implicit-GEMM conv vs
the vendor libraries PyTorch dispatches to (hipBLASLt for matmul, MIOpen for
conv), same random bf16 data, interleaved rounds in one process (guide §5.4
rule 24). Prints one JSON line per case; writes gpurun_out/bench_kernels.json.
"""
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_amd.ops._ext import load  # noqa: E402

C = load()
dev = torch.device("cuda", 0)


def timeit(fn, iters=20, rounds=5):
    fn()
    torch.cuda.synchronize()
    best = []
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        best.append(s.elapsed_time(e) / iters)
    best.sort()
    return best[len(best) // 2]


def gemm_cases():
    # (name, M, N, K): BERT-base T=4096 (B 32 x S 128), Llama-3-8B T=4096, ResNet 1x1 convs as GEMMs
    return [("bert_qkv", 4096, 2304, 768), ("bert_ffn1", 4096, 3072, 768), ("bert_ffn2", 4096, 768, 3072),
            ("llama_qkv", 4096, 6144, 4096), ("llama_gateup", 4096, 28672, 4096), ("llama_down", 4096, 4096, 14336),
            ("sq4096", 4096, 4096, 4096), ("sq8192", 8192, 8192, 8192),
            ("rn_l1_1x1", 802816, 64, 256), ("rn_l1_expand", 802816, 256, 64), ("rn_l4_1x1", 12544, 2048, 512)]


def main():
    out = []
    torch.manual_seed(0)
    for name, M, N, K in gemm_cases():
        a = torch.randn(M, K, device=dev).bfloat16()
        w = torch.randn(N, K, device=dev).bfloat16()
        flops = 2.0 * M * N * K
        t_ours = timeit(lambda: C.gemm(a, True, w, True, None, False, None, 0, None, False, 1.0, 1))
        t_ref = timeit(lambda: torch.matmul(a, w.t()))
        # dgrad (NN) and wgrad (TN, fp32 split-K)
        g = torch.randn(M, N, device=dev).bfloat16()
        t_dg = timeit(lambda: C.gemm(g, True, w, False, None, False, None, 0, None, False, 1.0, 1)) if N % 64 == 0 else None
        t_dg_ref = timeit(lambda: torch.matmul(g, w))
        t_wg = timeit(lambda: C.gemm(g, False, a, False, None, True, None, 0, None, False, 1.0, 0))
        t_wg_ref = timeit(lambda: torch.matmul(g.t(), a))
        r = {"kind": "gemm", "case": name, "M": M, "N": N, "K": K,
             "fwd_tflops": flops / t_ours / 1e9, "fwd_hipblaslt_tflops": flops / t_ref / 1e9,
             "dgrad_tflops": (flops / t_dg / 1e9) if t_dg else None, "dgrad_hipblaslt_tflops": flops / t_dg_ref / 1e9,
             "wgrad_tflops": flops / t_wg / 1e9, "wgrad_hipblaslt_tflops": flops / t_wg_ref / 1e9}
        print(json.dumps(r), flush=True)
        out.append(r)
        del a, w, g
        torch.cuda.empty_cache()
    # ResNet-50 3x3 convs at batch 256
    for name, (N, H, Cc, K, st) in {"rn_3x3_l1": (256, 56, 64, 64, 1), "rn_3x3_l2": (256, 28, 128, 128, 1),
                                    "rn_3x3_l3": (256, 14, 256, 256, 1), "rn_3x3_l4": (256, 7, 512, 512, 1),
                                    "rn_3x3_l2_s2": (256, 56, 128, 128, 2)}.items():
        x = torch.randn(N, H, H, Cc, device=dev).bfloat16()
        w = (torch.randn(K, 3, 3, Cc, device=dev) * 0.05).bfloat16()
        Ho = (H + 2 - 3) // st + 1
        flops = 2.0 * N * Ho * Ho * K * 9 * Cc
        t_ours = timeit(lambda: C.conv_fwd(x, w, st, 1, 1, False, None, 0, None))
        xc, wc = x.permute(0, 3, 1, 2), w.permute(0, 3, 1, 2)
        t_ref = timeit(lambda: F.conv2d(xc, wc, None, st, 1))
        dy = torch.randn(N, Ho, Ho, K, device=dev).bfloat16()
        dw = torch.empty(K, 3, 3, Cc, device=dev)
        t_wg = timeit(lambda: C.conv_wgrad(x, dy, dw, st, 1, 1, 0, False))
        dyc = dy.permute(0, 3, 1, 2)
        t_wg_ref = timeit(lambda: torch.ops.aten.convolution_backward(dyc, xc, wc, None, [st, st], [1, 1], [1, 1], False,
                                                                       [0, 0], 1, [False, True, False]))
        r = {"kind": "conv3x3", "case": name, "fwd_tflops": flops / t_ours / 1e9, "fwd_miopen_tflops": flops / t_ref / 1e9,
             "wgrad_tflops": flops / t_wg / 1e9, "wgrad_miopen_tflops": flops / t_wg_ref / 1e9}
        if st == 1:
            from k8s_amd.ops import conv as kc

            t_dg = timeit(lambda: kc.conv_bwd(dy, x, w, 1, 1, True, None))
            t_dg_ref = timeit(lambda: torch.ops.aten.convolution_backward(dyc, xc, wc, None, [1, 1], [1, 1], [1, 1],
                                                                           False, [0, 0], 1, [True, False, False]))
            r.update(dgrad_tflops=flops / t_dg / 1e9, dgrad_miopen_tflops=flops / t_dg_ref / 1e9)
        print(json.dumps(r), flush=True)
        out.append(r)
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(out, open("gpurun_out/bench_kernels.json", "w"), indent=1)


if __name__ == "__main__":
    main()
