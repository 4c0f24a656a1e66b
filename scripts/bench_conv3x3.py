"""Stride-1 3x3 convolutions of ResNet-50 at batch 1024: the staged-window kernel (conv3x3.hip) vs the implicit GEMM
(K8S_AMD_CONV3X3=0), forward with BN statistics, forward with bn1 normalised on load, and the data gradient;
interleaved rounds in one process, random operands.

    python scripts/bench_conv3x3.py [--batch 1024] [--rounds 3] > conv3x3.jsonl
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from k8s_amd.ops._ext import load  # noqa: E402

C_ = load()
dev = torch.device("cuda")


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    for H, C, K in [(56, 64, 64), (28, 128, 128), (14, 256, 256)]:
        N = a.batch
        x = (torch.rand(N, H, H, C, device=dev) * 2 - 1).bfloat16()
        w = ((torch.rand(K, 3, 3, C, device=dev) * 2 - 1) / (3 * C ** 0.5)).bfloat16()
        gy = (torch.rand(N, H, H, K, device=dev) * 2 - 1).bfloat16()
        w2 = C_.conv_dgrad_wtrans(w)
        stats = torch.zeros(C_.conv_stat_replicas, 2, K, device=dev)
        params = torch.stack([torch.rand(C, device=dev) + 0.5, torch.rand(C, device=dev) - 0.5]).contiguous()
        flop = 2.0 * N * H * H * K * 9 * C
        forms = {
            "fwd": lambda: C_.conv_fwd(x, w, 1, 1, 1, False, None, 0, stats),
            "fwd_bn_onload": lambda: C_.conv_fwd(x, w, 1, 1, 1, False, None, 0, stats, xform=params),
            "dgrad": lambda: C_.conv_fwd(gy, w2, 1, 1, 1, False, None, 0, None),
        }
        # arms: the staged-window kernel, the implicit GEMM (round 5 also timed a persistent pipelined form, "c3p":
        # profiles/r05_conv3x3_c3p_ab.jsonl)
        arms = {"staged": ("1", "0"), "implicit": ("0", "0")}
        # (round 6 timed the lean prologue against the round-5 kernel with these arms: profiles/r06_conv3x3_lean.jsonl,
        # "staged" = lean, "implicit" = round 5)
        for form, fn in forms.items():
            t = {k: [] for k in arms}
            for _ in range(a.rounds):
                for arm, (c3, c3p) in arms.items():
                    os.environ["K8S_AMD_CONV3X3"], os.environ["K8S_AMD_C3P"] = c3, c3p
                    t[arm].append(timeit(fn))
            rec = {"shape": [N, H, H, C, K], "form": form}
            for arm in arms:
                us = min(t[arm]) * 1e3
                rec[arm + "_us"] = round(us, 1)
                rec[arm + "_tf"] = round(flop / us / 1e6)
            rec["staged_vs_implicit"] = round(rec["implicit_us"] / rec["staged_us"], 3)
            print(json.dumps(rec), flush=True)
        del x, w, gy, w2
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
