"""Per-rank update cost of the ZeRO-1 service on one GPU, Llama-3-8B-sized flat buffers (8.03 B parameters):

    full      fused Adam over the whole model + refresh_lowp (the bf16 copy rebuilt from the fp32 master): what one
              rank paid per step before sharding, and the copy the round-3 sharded path still paid after its fp32
              all-gather of the master
    sharded   fused Adam over this rank's 1/world of every 64 MB bucket, writing its bf16 slice in the same pass --
              the bf16 pull (an all-gather, not timed here: it runs on the wire) replaces the refresh copy

    python scripts/bench_zero_update.py [--params 8.03e9] [--world 8]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from k8s_amd.ops.optim import FusedAdam  # noqa: E402
from k8s_amd.parallel.flat import ALIGN, ParamStore, init_const  # noqa: E402


def timeit(fn, reps=5):
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
    ap.add_argument("--params", type=float, default=8.03e9)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--bucket-mb", type=float, default=256.0)
    a = ap.parse_args()
    dev = torch.device("cuda")
    n = int(a.params) // (a.world * ALIGN) * (a.world * ALIGN)
    store = ParamStore()
    store.new("flat", (n,), init_const(0.01))
    store.finalize(dev, pad_to=a.world * ALIGN)
    store.grad.fill_(1e-3)
    cap = int(a.bucket_mb * 2 ** 20 / 4) // (a.world * ALIGN) * (a.world * ALIGN)
    ranges, hi = [], store.total
    while hi > 0:  # the service's buckets (from the end), this rank's 1/world slice of each
        lo = max(0, hi - cap)
        k = (hi - lo) // a.world
        ranges.append((lo + 3 * k, lo + 4 * k))  # rank 3's slice
        hi = lo
    full = FusedAdam(store, lr=1e-4)
    t_full = timeit(lambda: (full.step(grad_scale=1.0 / a.world), store.refresh_lowp()))
    del full
    torch.cuda.empty_cache()
    sh = FusedAdam(store, lr=1e-4)
    sh.shard(ranges)
    t_sh = timeit(lambda: sh.step(grad_scale=1.0 / a.world, ranges=ranges))
    print(json.dumps({"params": n, "world": a.world, "full_adam_plus_refresh_ms": round(t_full, 2),
                      "sharded_adam_ms": round(t_sh, 2), "ratio": round(t_full / t_sh, 2)}), flush=True)


if __name__ == "__main__":
    main()
