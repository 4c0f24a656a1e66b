"""1x1-convolution forward shapes of ResNet-50 b1024: our conv_fwd (with / without the BN-statistics epilogue) vs
our generic GEMM entry and torch.matmul (hipBLASLt), same process. One JSON line per shape."""
import json
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from k8s_amd.ops._ext import load  # noqa: E402

C_ = load()
d = torch.device("cuda")


def timed(f, reps=20):
    f()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            f()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) / reps)
    return round(best * 1e3, 1)


N = 1024
for H, C, K in [(56, 256, 64), (56, 64, 256), (28, 512, 128), (28, 128, 512), (14, 1024, 256), (14, 256, 1024),
                (7, 2048, 512), (7, 512, 2048)]:
    x = torch.randn(N, H, H, C, device=d, dtype=torch.bfloat16)
    w = (torch.randn(K, 1, 1, C, device=d) * C ** -0.5).bfloat16()
    st = torch.zeros(C_.conv_stat_replicas, 2, K, device=d)
    xfp = torch.cat([torch.rand(C, device=d) + 0.5, torch.randn(C, device=d) * 0.1]).contiguous()
    x2, w2 = x.view(-1, C), w.view(K, C)
    M = x2.shape[0]
    r = {"MNK": [M, K, C],
         "conv_stats": timed(lambda: C_.conv_fwd(x, w, 1, 0, 1, False, None, 0, st)),
         "conv_nostats": timed(lambda: C_.conv_fwd(x, w, 1, 0, 1, False, None, 0, None)),
         "conv_xf_stats": timed(lambda: C_.conv_fwd(x, w, 1, 0, 1, False, None, 0, st, xform=xfp)),
         "gemm": timed(lambda: C_.gemm(x2, True, w2, True, None, False, None, 0, None, False, 1.0, 1)),
         "blas": timed(lambda: torch.matmul(x2, w2.t()))}
    # data gradient of the same layer: dx[M, C] = dy[M, K] . w[K, C] (reduction K), plain and onto a masked addend
    gy = torch.randn(M, K, device=d, dtype=torch.bfloat16)
    dy = torch.randn(M, C, device=d, dtype=torch.bfloat16)
    mask = torch.randint(0, 256, (M * C // 8,), device=d, dtype=torch.uint8)
    out = torch.empty(M, C, device=d, dtype=torch.bfloat16)
    r["dgrad"] = timed(lambda: C_.gemm(gy, True, w2, False, None, False, None, 0, None, False, 1.0, 1))
    r["dgrad_masked"] = timed(lambda: C_.gemm(gy, True, w2, False, out, False, None, 0, None, True, 1.0, 1, dy, mask))
    r["dgrad_blas"] = timed(lambda: torch.matmul(gy, w2))
    r["hbm_floor"] = round((M * C + M * K) * 2 / 8e6, 1)
    r["short_fwd"] = bool(C_.gemm_short_ok(M, K, C))
    r["short_dgrad"] = bool(C_.gemm_short_ok(M, C, K))
    del gy, dy, mask, out
    print(json.dumps(r), flush=True)
    del x, w, x2, w2
    torch.cuda.empty_cache()
