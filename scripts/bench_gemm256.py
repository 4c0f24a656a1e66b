"""Large-GEMM A/B: the 256 x 256 phased MFMA kernel (gemm256.hip) vs hipBLASLt (torch.mm) vs the 128 x 128 kernel,
interleaved rounds in ONE process on uniform random [-1, 1) bf16 operands (cdna_hip_programming.md §5.4 rules 24/25).

Every Llama-3-8B (M = 4096 tokens) and BERT-base (M = 8192 tokens) linear product in its three forms:
    fwd   y  = x . W^T   (A K-major,  B K-major)     torch: x @ W.t()
    dgrad dx = g . W     (A K-major,  B N-major)     torch: g @ W
    wgrad dW = g^T . x   (A M-major,  B N-major)     torch: g.t() @ x   (fp32 out, split-K chosen as in training)

    python scripts/bench_gemm256.py [--rounds 5] [--only llama|bert|square] > gemm256.jsonl
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_amd.ops._ext import load  # noqa: E402

C = load()
dev = torch.device("cuda")

# (name, tokens M, out features N, in features K)
LAYERS = {
    "llama": [("qkv", 4096, 6144, 4096), ("o", 4096, 4096, 4096), ("gate_up", 4096, 28672, 4096),
              ("down", 4096, 4096, 14336), ("lm_head", 4096, 128256, 4096)],
    "bert": [("qkv", 8192, 2304, 768), ("o", 8192, 768, 768), ("ffn1", 8192, 3072, 768), ("ffn2", 8192, 768, 3072)],
    "square": [("sq4096", 4096, 4096, 4096), ("sq8192", 8192, 8192, 8192)],
}


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


def rnd(*shape):
    return (torch.rand(*shape, device=dev) * 2 - 1).bfloat16()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--only", default=None)
    ap.add_argument("--forms", default="fwd,dgrad,wgrad", help="comma list of fwd,dgrad,wgrad")
    ap.add_argument("--variants", nargs="*", default=[], help="extra ENV=VALUE[,ENV=VALUE] arms, e.g. K8S_AMD_GEMM256=0 (force the 128 x 128 kernel)")
    a = ap.parse_args()
    groups = [a.only] if a.only else list(LAYERS)
    for grp in groups:
        for name, M, N, K in LAYERS[grp]:
            x, w, g = rnd(M, K), rnd(N, K), rnd(M, N)
            dw = torch.empty(N, K, device=dev)
            forms = {
                "fwd": (lambda: C.gemm(x, True, w, True, None, False, None, 0, None, False, 1.0, 1),
                        lambda: x @ w.t(), 2.0 * M * N * K),
                "dgrad": (lambda: C.gemm(g, True, w, False, None, False, None, 0, None, False, 1.0, 1),
                          lambda: g @ w, 2.0 * M * N * K),
                "wgrad": (lambda: C.gemm(g, False, x, False, dw, True, None, 0, None, False, 1.0, 0),
                          lambda: g.t() @ x, 2.0 * M * N * K),
            }
            for form, (ours, blas, flop) in forms.items():
                if form not in a.forms.split(","):
                    continue
                to, tb, tv = [], [], {v: [] for v in a.variants}
                for _ in range(a.rounds):
                    to.append(timeit(ours))
                    tb.append(timeit(blas))
                    for v in a.variants:  # ENV=VALUE[,ENV=VALUE] A/B arms of our kernel, same process
                        saved = {}
                        for kv in v.split(","):
                            k_, v_ = kv.split("=")
                            saved[k_] = os.environ.get(k_)
                            os.environ[k_] = v_
                        tv[v].append(timeit(ours))
                        for k_, old in saved.items():
                            if old is None:
                                os.environ.pop(k_)
                            else:
                                os.environ[k_] = old
                ref = blas().float()
                got = ours().float()
                err = ((got - ref).norm() / ref.norm()).item()
                o, b = min(to), min(tb)
                rec = {"group": grp, "layer": name, "form": form, "MNK": [M, N, K],
                       "ours_us": round(o * 1e3, 1), "blas_us": round(b * 1e3, 1),
                       "ours_tf": round(flop / o / 1e9), "blas_tf": round(flop / b / 1e9),
                       "speedup": round(b / o, 3), "relerr": round(err, 5)}
                for v, ts in tv.items():
                    rec["tf[%s]" % v] = round(flop / min(ts) / 1e9)
                print(json.dumps(rec), flush=True)
            del x, w, g, dw
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
