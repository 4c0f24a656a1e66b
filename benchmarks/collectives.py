#!/usr/bin/env python3
"""RCCL collective bandwidth over xGMI: all-reduce / reduce-scatter / all-gather / all-to-all busbw.

BASELINE config 4 reports "all-reduce busbw" next to Llama-3-8B tokens/s; config 2's
1/2/4/8 ResNet scaling is bounded by the same number. Sizes sweep the gradient-bucket
range the reducers use (``parallel/ddp.py``, ``parallel/ps.py``: 64 MB default buckets,
102 MB of fp32 ResNet-50 gradients, 16 GB of bf16 Llama-3-8B gradients).

Bus bandwidth follows the usual convention so numbers are comparable with rccl-tests:
    all_reduce      busbw = algbw * 2(n-1)/n
    reduce_scatter  busbw = algbw * (n-1)/n      (algbw over the full input)
    all_gather      busbw = algbw * (n-1)/n      (algbw over the full output)
    all_to_all      busbw = algbw * (n-1)/n
On a fully connected 8x MI355X xGMI mesh each GPU has 7 links of ~153 GB/s/direction;
a single ring uses one link per direction, so RCCL needs multiple channels/rings to
approach the 7-link aggregate -- this benchmark shows where the buckets land.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        benchmarks/collectives.py --sizes-mb 1,16,64,256,1024
    python -m torch.distributed.run --nproc-per-node 2 ... benchmarks/collectives.py --device cpu  (gloo)

Rank 0 prints one JSON line per (op, size) with the MAX time over ranks.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from k8s_amd.parallel import dist as kdist  # noqa: E402

OPS = ("all_reduce", "reduce_scatter", "all_gather", "all_to_all")


def bus_factor(op: str, n: int) -> float:
    if n <= 1:
        return 1.0
    return 2.0 * (n - 1) / n if op == "all_reduce" else (n - 1) / n


def run_op(op, buf, out, n):
    if op == "all_reduce":
        dist.all_reduce(buf)
    elif op == "reduce_scatter":
        dist.reduce_scatter_tensor(out, buf)
    elif op == "all_gather":
        dist.all_gather_into_tensor(buf, out)
    elif op == "all_to_all":
        dist.all_to_all_single(out, buf)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--sizes-mb", default="1,4,16,64,256,1024")
    ap.add_argument("--ops", default=",".join(OPS))
    ap.add_argument("--dtype", default="bf16", choices=("bf16", "fp32"))
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--device", default="auto", choices=("auto", "cuda", "cpu"))
    a = ap.parse_args(argv)

    use_cuda = torch.cuda.is_available() and a.device != "cpu"
    info = kdist.init_process_group(backend=None if use_cuda else "gloo")
    n, rank = info.world_size, info.rank
    dev = torch.device("cuda", info.local_rank) if use_cuda else torch.device("cpu")
    dtype = torch.bfloat16 if (a.dtype == "bf16" and use_cuda) else torch.float32
    esz = torch.tensor([], dtype=dtype).element_size()
    sync = torch.cuda.synchronize if use_cuda else (lambda: None)
    for op in a.ops.split(","):
        for mb in (float(s) for s in a.sizes_mb.split(",")):
            numel = max(n, int(mb * 1024 * 1024 / esz) // n * n)
            buf = torch.ones(numel, device=dev, dtype=dtype)
            out = torch.empty(numel // n if op in ("reduce_scatter", "all_gather") else numel, device=dev,
                              dtype=dtype)
            if op == "all_to_all":
                out = torch.empty_like(buf)
            if n == 1 and op != "all_reduce":
                continue
            for _ in range(a.warmup):
                run_op(op, buf, out, n)
            sync()
            kdist.barrier()
            t0 = time.perf_counter()
            for _ in range(a.iters):
                run_op(op, buf, out, n)
            sync()
            dt = kdist.all_reduce_max((time.perf_counter() - t0) / a.iters, dev)
            nbytes = numel * esz
            algbw = nbytes / dt / 1e9
            if rank == 0:
                print(json.dumps({"op": op, "bytes": nbytes, "n": n, "dtype": str(dtype).split(".")[-1],
                                  "backend": dist.get_backend() if dist.is_initialized() else "none",
                                  "us": round(dt * 1e6, 1), "algbw_GBs": round(algbw, 4),
                                  "busbw_GBs": round(algbw * bus_factor(op, n), 4)}), flush=True)
            del buf, out
    kdist.destroy()


if __name__ == "__main__":
    main()
