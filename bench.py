#!/usr/bin/env python3
"""Headline benchmark: ResNet-50 training images/sec on N MI355X GPUs.

Metric and config come from BASELINE.json ("images/sec ResNet-50 TfJob at
1/2/4/8 MI355X"): ResNet-50 v1.5, synthetic ImageNet (224x224x3, 1000
classes, random-init weights -- no datasets or checkpoints are reachable),
bf16 compute with fp32 master weights/BN statistics, SGD+momentum (fused HIP
kernel), data parallel with bucketed RCCL all-reduce overlapped with
backward. Per-GPU batch (default 3072, 113 GB of the 288 GB HBM) is fixed as N grows (weak scaling).

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Rank 0 prints ONE JSON line; ``value`` is the whole-job images/sec computed
from the MAX per-rank wall time over exactly K timed steps bracketed by a
barrier + device synchronize on both sides.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

# RCCL / HIP environment, set before anything initialises the GPU (the first HIP call happens in
# kdist.init_process_group -> torch.cuda.set_device). The KFD on the MI355X hosts this runs on only supports
# dmabuf-based peer memory: without HSA_ENABLE_IPC_MODE_LEGACY=0 RCCL's intra-node transport and CUDA-IPC tensor
# sharing fail with `hipIpcGetMemHandle: invalid argument` (observed on these hosts; the same requirement is in
# charts/tf-job-operator/values.yaml `ipcModeLegacy` and the task environment notes). setdefault: an operator-set
# value wins. RCCL's channel count is left to its own MI3xx tuning (charts/... `minChannels` is a knob, not a
# requirement).
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from k8s_amd.models.resnet import resnet50  # noqa: E402
from k8s_amd.ops import nn as K  # noqa: E402
from k8s_amd.ops.optim import FusedSGD  # noqa: E402
from k8s_amd.parallel import dist as kdist  # noqa: E402
from k8s_amd.parallel.ddp import GradReducer  # noqa: E402
from k8s_amd.parallel.flat import ParamStore  # noqa: E402

BASELINE_VALUE = None  # BASELINE.json "published": {} -- the reference publishes no number


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    # 3072 images per GPU (113 GB peak of 288 GB HBM, reported as peak_mem_gb): one MI355X box, round 5 tree,
    # 14,870 img/s vs 14,712 at 2048 and 14,287 at 1024 (profiles/r05_batch_sweep.jsonl) -- the 7x7 / 14x14
    # layers and the per-launch prologues amortise over more rows; >= 2048 exercises the chunked short-K launches
    # (tests/test_resnet_gpu.py duplicated-half-batch check at 2048 / 3072)
    ap.add_argument("--batch", type=int, default=3072, help="per-GPU batch")
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--bucket-mb", type=float, default=64.0)
    ap.add_argument("--grad-comm", choices=["fp32", "bf16"], default="fp32",
                    help="gradient all-reduce transport (bf16: all-to-all + fp32 owner sum + all-gather)")
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--profile-steps", type=int, default=0, help="(internal) roctx-free short run")
    ap.add_argument("--force-dist", action="store_true",
                    help="create the process group and run the gradient transport even at world 1 (RCCL on one GPU)")
    return ap.parse_args(argv)


def _launch_local_ranks(a, argv) -> int:
    """``--gpus N`` (N > 1) without a launcher: start N local rank processes ourselves, one per GPU, BEFORE this
    process touches the GPU (the pattern of trainer/runner.py ``_run_replica_children``). Each child gets
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT like torch.distributed.run would set; rank 0's JSON
    line goes straight to our stdout. Returns the first non-zero child exit code (0 when all succeed); when one rank
    fails the others get a grace period, then SIGTERM (they would otherwise wait in a collective forever)."""
    import signal
    import subprocess

    from k8s_amd.fakeapi.server import free_port

    port = free_port()
    script = os.path.abspath(__file__)
    argv = list(sys.argv[1:] if argv is None else argv)
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus), LOCAL_WORLD_SIZE=str(a.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script] + argv, env=env))

    def forward(signum, _frame):
        for p in procs:
            if p.poll() is None:
                p.send_signal(signum)

    signal.signal(signal.SIGTERM, forward)
    codes = [None] * len(procs)
    deadline = None
    while any(c is None for c in codes):
        for i, p in enumerate(procs):
            if codes[i] is None and p.poll() is not None:
                codes[i] = 128 - p.returncode if p.returncode < 0 else p.returncode
                if codes[i] != 0 and deadline is None:
                    deadline = time.time() + 30.0
        if deadline is not None and time.time() > deadline:
            forward(signal.SIGTERM, None)
            deadline = float("inf")
        time.sleep(0.05)
    bad = [c for c in codes if c != 0]
    return bad[0] if bad else 0


def _comm_record(n, dev):
    """backend / RCCL version / world size as the live process group reports them (not as requested)."""
    import torch.distributed as tdist

    rec = {"backend": "none", "world_size": 1, "rccl_version": None}
    if tdist.is_available() and tdist.is_initialized():
        rec["backend"] = str(tdist.get_backend())
        rec["world_size"] = int(tdist.get_world_size())
    if dev.type == "cuda":
        try:
            v = torch.cuda.nccl.version()
            rec["rccl_version"] = ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
        except Exception as e:  # noqa: BLE001 -- recorded, not fatal
            rec["rccl_version"] = "unavailable: %s" % e
        rec["device"] = torch.cuda.get_device_name(dev)
        try:
            from k8s_amd.ops._ext import load as _load_ext

            rec["planner_cus"] = int(_load_ext().planner_cus())
        except Exception:  # noqa: BLE001
            pass
    return rec


def main(argv=None):
    a = parse(argv)
    if a.gpus > 1 and "RANK" not in os.environ and "WORLD_SIZE" not in os.environ:
        return _launch_local_ranks(a, argv)
    info = kdist.init_process_group(force=a.force_dist)
    n = info.world_size
    if n != a.gpus:
        # fail closed: a number measured on a different world than the one asked for must not be reported
        print("error: --gpus %d but the process group has world size %d" % (a.gpus, n), file=sys.stderr)
        kdist.destroy()
        return 2
    dev = torch.device("cuda", info.device_index) if torch.cuda.is_available() else torch.device("cpu")
    torch.manual_seed(1234 + info.rank)

    store = ParamStore()
    model = resnet50(store).finalize(dev)
    model.train()
    # DP replicas start from identical weights (same seed in finalize); broadcast for safety
    if n > 1:
        torch.distributed.broadcast(store.master, 0)
        store.refresh_lowp()
    reducer = GradReducer(store, bucket_mb=a.bucket_mb, enabled=(n > 1 or a.force_dist),
                          comm_dtype=torch.bfloat16 if a.grad_comm == "bf16" else torch.float32)
    opt = FusedSGD(store, lr=a.lr, momentum=0.9, weight_decay=5e-5, nesterov=False)
    # what the collectives actually ran on, read from the process group after its first collective (the broadcast
    # above): the driver's multi-GPU record must show by itself that RCCL initialised with every rank
    comm = _comm_record(n, dev)
    # step-0 transport self-check (untimed): one gradient bucket through the configured transport vs a plain fp32
    # all_reduce of the same data; a mismatch beyond the transport's rounding fails the run before any number
    check = reducer.self_check()
    if not check["ok"]:
        if info.rank == 0:
            print("error: gradient transport self-check failed: %s" % json.dumps(check), file=sys.stderr)
        kdist.destroy()
        return 3

    dtype = torch.bfloat16 if dev.type == "cuda" else torch.float32
    images = torch.randn(a.batch, a.image, a.image, 3, device=dev, dtype=dtype)
    x = model.prepare_input(images).contiguous()
    labels = torch.randint(0, 1000, (a.batch,), device=dev)

    # comm_exposed_ms: per step, the time from the end of backward to the end of reducer.finish() (the collective
    # work backward did not hide). On the GPU from events recorded on the compute stream (no host sync inside the
    # timed loop; read after it); on the CPU (gloo, synchronous) from the host clock.
    marks = []

    def step(timed=False):
        reducer.begin_step()
        logits = model(x)
        loss = K.cross_entropy(logits, labels)
        loss.backward()
        if timed and dev.type == "cuda":
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            reducer.finish()
            e1.record()
            marks.append((e0, e1))
        elif timed:
            t = time.perf_counter()
            reducer.finish()
            marks.append(time.perf_counter() - t)
        else:
            reducer.finish()
        opt.step(grad_scale=reducer.grad_scale)
        return loss

    for i in range(a.warmup):
        loss = step()
        if info.rank == 0:  # progress on stderr (the first step JIT-loads kernels)
            print("warmup step %d/%d issued" % (i + 1, a.warmup), file=sys.stderr, flush=True)
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    sync()
    kdist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step(timed=True)
    sync()
    kdist.barrier()
    sync()
    dt = time.perf_counter() - t0
    dt_max = kdist.all_reduce_max(dt, dev)
    if dev.type == "cuda":
        exposed = [e0.elapsed_time(e1) for e0, e1 in marks]
    else:
        exposed = [1000.0 * t for t in marks]
    exposed_ms = kdist.all_reduce_max(sum(exposed) / max(1, len(exposed)), dev)
    final_loss = float(loss.detach().float().item())
    # data-parallel sanity (outside the timed region): every replica must hold the same weights
    csum = float(store.master.double().sum().item())
    identical = kdist.all_reduce_max(csum, dev) == -kdist.all_reduce_max(-csum, dev)
    ips = n * a.batch * a.steps / dt_max
    if info.rank == 0:
        out = {
            "metric": "images/sec ResNet-50 TfJob (train, synthetic ImageNet)",
            "value": round(ips, 2),
            "unit": "images/s",
            "n_gpus": n,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1000.0 * dt_max / a.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (ips / BASELINE_VALUE) if BASELINE_VALUE else None,
            "dtype": "bf16" if dev.type == "cuda" else "fp32",
            "data": "synthetic (random %dx%dx3 images, random labels, random-init weights)" % (a.image, a.image),
            "config": {
                "model": "resnet50-v1.5",
                "global_batch": n * a.batch,
                "per_gpu_batch": a.batch,
                "seq_len": None,
                "image_size": a.image,
                "parallelism": "dp%d" % n,
                "optimizer": "fused SGD momentum 0.9 (HIP)",
                "bucket_mb": a.bucket_mb,
            },
            "final_loss": round(final_loss, 4),
            "replicas_identical": identical,
            "comm_exposed_ms": round(exposed_ms, 3),
            "comm": comm,
            "transport_check": check,
            "grad_comm_fallbacks": dict(reducer.fallbacks),
            "peak_mem_gb": round(torch.cuda.max_memory_allocated(dev) / 2**30, 1) if dev.type == "cuda" else None,
        }
        print(json.dumps(out), flush=True)
        if dev.type == "cuda":
            from k8s_amd.ops import conv, gemm

            print("conv paths: %s" % json.dumps(conv.STATS), file=sys.stderr)
            print("gemm fallbacks: %s" % json.dumps(gemm.FALLBACKS), file=sys.stderr)
    kdist.destroy()


if __name__ == "__main__":
    sys.exit(main() or 0)
