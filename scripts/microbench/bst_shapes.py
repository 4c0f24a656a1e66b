"""Per-shape cost of the BatchNorm-backward-sums epilogues on the tile kernel (gemm.hip BST fast path, mask kind)
against the plain data gradient each replaced, on the ResNet-50 b3072 shapes: the stem pool's downsample dgrad
(accumulate, N = 64), the stage-3 / 4 downsample blocks' outputs read by the next conv1 (masked addend, two BNs) and
the stage-4 identity block (masked addend, one BN). One JSON line per shape."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from k8s_amd.ops._ext import load  # noqa: E402


def timed(fn, reps=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    C = load()
    d = torch.device("cuda")
    R = C.conv_stat_replicas
    b = int(os.environ.get("BST_BATCH", "3072"))
    shapes = [("pool_down", b * 56 * 56, 64, 256, "acc", False), ("s3b0_out", b * 14 * 14, 1024, 256, "mask", True),
              ("s4b0_out", b * 49, 2048, 512, "mask", True), ("s4b1_out", b * 49, 2048, 512, "mask", False)]
    for name, M, N, K, kind, dual in shapes:
        gy = torch.randn(M, K, device=d).bfloat16()
        w = (torch.randn(K, N, device=d) * 0.05).bfloat16()
        add = torch.randn(M, N, device=d).bfloat16()
        amask = torch.randint(0, 256, (M * N // 8,), device=d, dtype=torch.uint8)
        x = torch.randn(M, N, device=d).bfloat16()
        x2 = torch.randn(M, N, device=d).bfloat16() if dual else None
        mask = torch.randint(0, 256, (M * N // 8,), device=d, dtype=torch.uint8)
        mean = torch.zeros(N, device=d)
        sums = torch.zeros(R, 2, N, device=d)
        sums2 = torch.zeros(R, 2, N, device=d) if dual else None
        out = torch.empty(M, N, device=d).bfloat16()
        if kind == "acc":
            plain = lambda: C.gemm(gy, True, w, False, out, False, None, 0, None, True, 1.0, 1)  # noqa: E731
            fused = lambda: C.gemm_dgrad_bnstats_mask(gy, w, out, x, mask, mean, sums)  # noqa: E731
        else:
            plain = lambda: C.gemm(gy, True, w, False, out, False, None, 0, None, True, 1.0, 1,  # noqa: E731
                                   add_src=add, add_mask=amask)
            fused = lambda: C.gemm_dgrad_bnstats_mask(gy, w, out, x, mask, mean, sums, add, amask,  # noqa: E731
                                                      x2, mean if dual else None, sums2)
        tp, tf = timed(plain), timed(fused)
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "dual": dual, "plain_us": round(tp, 1),
                          "fused_us": round(tf, 1)}), flush=True)
        del gy, w, add, amask, x, x2, mask, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
