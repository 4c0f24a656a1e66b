"""Data-parallel strategies on CPU with gloo, 2 and 4 ranks (the RCCL code paths, minus the device).

* all-reduce (``GradReducer``) vs the sharded parameter service (``ShardedParameterService``, reduce-scatter
  push / ZeRO-1 owner update / all-gather pull): same weights and optimizer state; bit-for-bit at 2 ranks
  (a + b == b + a), to rounding at 4 (the two collectives sum in different orders).
* bf16 gradient transport (all-to-all reduce-scatter + fp32 accumulation): close to the fp32 result, and the
  fp32 summation is what keeps it close (a bf16 running sum would not be).
* ZeRO-1: each rank holds 1/world of the optimizer moments.
* non-finite gradients under gradient clipping skip the step on every rank, leaving all state bit-identical.
"""
import os
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from k8s_amd.fakeapi.server import free_port

SHAPES = [(64, 33), (129,), (7, 5, 3), (256,), (16, 16), (1000,)]


def _grads(rank, step, shapes):
    g = torch.Generator().manual_seed(1000 * step + 17 * rank + 3)
    return [torch.randn(s, generator=g) * (1.0 + rank) for s in shapes]


def _worker(rank, world, port, strategy, comm, opt_name, steps, out_dir, nan_step, clip=10.0, pull="auto"):
    from k8s_amd.ops.optim import FusedAdam, FusedSGD
    from k8s_amd.parallel.ddp import GradReducer
    from k8s_amd.parallel.flat import ALIGN, ParamStore, init_normal
    from k8s_amd.parallel.ps import ShardedParameterService

    torch.set_num_threads(1)
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    store = ParamStore()
    params = [store.new("p%d" % i, s, init_normal(0.5), decay=(i % 2 == 0), lowp=(i % 3 != 2)) for i, s in enumerate(SHAPES)]
    store.finalize("cpu", pad_to=world * ALIGN, seed=5)
    if opt_name == "sgd":
        opt = FusedSGD(store, lr=0.05, momentum=0.9, weight_decay=1e-3, max_grad_norm=clip)
    else:
        opt = FusedAdam(store, lr=0.01, weight_decay=0.01, max_grad_norm=clip)
    dtype = torch.bfloat16 if comm == "bf16" else torch.float32
    if strategy == "ps":
        svc = ShardedParameterService(store, opt, bucket_mb=0.002, comm_dtype=dtype, pull=pull)  # several buckets
        begin, finish = svc.begin_step, (lambda: svc.step())
    else:
        red = GradReducer(store, bucket_mb=0.002, comm_dtype=dtype)
        begin = red.begin_step

        def finish():
            red.finish()
            opt.step(grad_scale=red.grad_scale)
        svc = None
    for step in range(steps):
        begin()
        gs = _grads(rank, step, SHAPES)
        if step == nan_step and rank == world - 1:
            gs[2][0, 0, 0] = float("nan")
        for p, g in reversed(list(zip(params, gs))):  # backward order
            store.deposit(p, g)
        finish()
    stale_ok = True
    if svc is not None and svc.pull == "lowp" and world > 1:
        # before sync_master: the bf16 copy is whole, the fp32 master current on this rank's owned slices and on the
        # fp32-read (lowp=False) parameters only
        store.wait_pending()
        ref_half = store.half.clone()
        svc.sync_master()
        stale_ok = torch.equal(ref_half, store.half) and torch.equal(store.half, store.master.to(torch.bfloat16))
    full = svc.gather_state() if svc is not None else None
    if rank == 0:
        sd = opt.state_dict(full)
        torch.save({"master": store.master.clone(), "half": store.half.float().clone(),
                    **{k: v.clone() for k, v in sd.items() if torch.is_tensor(v)},
                    "state_numel": opt.state_numel(), "total": store.total, "stale_ok": stale_ok},
                   os.path.join(out_dir, "%s_%s_%s.pt" % (strategy, comm, opt_name)))
    dist.barrier()
    dist.destroy_process_group()


def _run(world, strategy, comm, opt_name, steps=4, nan_step=-1, clip=10.0, pull="auto"):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, free_port(), strategy, comm, opt_name, steps, d, nan_step, clip, pull),
                 nprocs=world)
        return torch.load(os.path.join(d, "%s_%s_%s.pt" % (strategy, comm, opt_name)), weights_only=True)


def _reference(world, opt_name, steps):
    """Single-process ground truth: the fp32 sum of every rank's gradient, one optimizer over everything."""
    from k8s_amd.ops.optim import FusedAdam, FusedSGD
    from k8s_amd.parallel.flat import ALIGN, ParamStore, init_normal

    store = ParamStore()
    params = [store.new("p%d" % i, s, init_normal(0.5), decay=(i % 2 == 0), lowp=(i % 3 != 2)) for i, s in enumerate(SHAPES)]
    store.finalize("cpu", pad_to=world * ALIGN, seed=5)
    if opt_name == "sgd":
        opt = FusedSGD(store, lr=0.05, momentum=0.9, weight_decay=1e-3, max_grad_norm=10.0)
    else:
        opt = FusedAdam(store, lr=0.01, weight_decay=0.01, max_grad_norm=10.0)
    for step in range(steps):
        store.begin_step()
        tot = [sum(_grads(r, step, SHAPES)[i] for r in range(world)) for i in range(len(SHAPES))]
        for p, g in zip(params, tot):
            store.deposit(p, g)
        opt.step(grad_scale=1.0 / world)
    return store.master.clone()


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("opt_name", ["sgd", "adam"])
def test_allreduce_and_sharded_ps_agree(world, opt_name):
    a = _run(world, "allreduce", "fp32", opt_name)
    b = _run(world, "ps", "fp32", opt_name)
    keys = ["master", "half"] + (["momentum_buffer"] if opt_name == "sgd" else ["exp_avg", "exp_avg_sq"])
    for k in keys:
        if world == 2:
            assert torch.equal(a[k], b[k]), k  # same two-term sums: bit-for-bit
        else:
            torch.testing.assert_close(a[k], b[k], rtol=1e-6, atol=1e-7, msg=k)
    torch.testing.assert_close(a["master"], _reference(world, opt_name, 4), rtol=1e-5, atol=1e-6)
    # ZeRO-1: the sharded run kept 1/world of the moments per rank
    n_state = 1 if opt_name == "sgd" else 2
    assert a["state_numel"] == n_state * a["total"]
    assert b["state_numel"] == n_state * b["total"] // world


@pytest.mark.parametrize("strategy", ["allreduce", "ps"])
def test_bf16_gradient_transport_close_to_fp32(strategy):
    world = 4
    ref = _reference(world, "sgd", 4)
    b = _run(world, strategy, "bf16", "sgd")
    f = _run(world, strategy, "fp32", "sgd")
    err_b = (b["master"] - ref).abs().max().item()
    err_f = (f["master"] - ref).abs().max().item()
    assert err_f < 1e-5
    assert err_b < 5e-3, err_b  # one bf16 rounding per contribution, fp32 accumulation


@pytest.mark.parametrize("strategy", ["allreduce", "ps"])
def test_nonfinite_gradient_skips_step_everywhere(strategy):
    """A NaN in one rank's gradient at the last step: the clip factor is 0 and the update is skipped, so the
    final state equals a run that stopped one step earlier (bit for bit)."""
    a = _run(2, strategy, "fp32", "adam", steps=4, nan_step=3)
    b = _run(2, strategy, "fp32", "adam", steps=3)
    for k in ("master", "exp_avg", "exp_avg_sq"):
        assert torch.equal(a[k], b[k]), k


def _reference_bf16(world, opt_name, steps, round_sum, clip=None):
    """Ground truth of the bf16 transport: every rank's contribution rounded to bf16 once, summed in fp32 in RANK
    ORDER (what slice_sum does on the owner); ``round_sum``: the all-reduce strategy also rounds the reduced slice
    to bf16 for its all-gather."""
    from k8s_amd.ops.optim import FusedAdam, FusedSGD
    from k8s_amd.parallel.flat import ALIGN, ParamStore, init_normal

    store = ParamStore()
    params = [store.new("p%d" % i, s, init_normal(0.5), decay=(i % 2 == 0), lowp=(i % 3 != 2)) for i, s in enumerate(SHAPES)]
    store.finalize("cpu", pad_to=world * ALIGN, seed=5)
    if opt_name == "sgd":
        opt = FusedSGD(store, lr=0.05, momentum=0.9, weight_decay=1e-3, max_grad_norm=clip)
    else:
        opt = FusedAdam(store, lr=0.01, weight_decay=0.01, max_grad_norm=clip)
    for step in range(steps):
        store.begin_step()
        per = [_grads(r, step, SHAPES) for r in range(world)]
        for i, p in enumerate(params):
            acc = torch.zeros(p.shape)
            for r in range(world):
                acc = acc + per[r][i].to(torch.bfloat16).float()
            if round_sum:
                acc = acc.to(torch.bfloat16).float()
            store.deposit(p, acc)
        opt.step(grad_scale=1.0 / world)
    return store.master.clone()


@pytest.mark.parametrize("world", [3, 4, 8])
@pytest.mark.parametrize("strategy", ["allreduce", "ps"])
def test_bf16_transport_bit_exact_against_rank_order_reference(world, strategy):
    """4- and 8-rank runs bit-exact against the single-process reference; 3 ranks (a world
    that does not divide the 64-element bucket alignment) take the zero-padded exchange, not an fp32 fallback. The bf16
    transport sums in a fixed (rank) order, so its result is reproducible to the bit: Adam, 4 steps. (No gradient
    clipping here: the sharded clip norm is an all-reduce of per-shard partial sums, whose order differs from a
    single-process norm in the last bit.)"""
    got = _run(world, strategy, "bf16", "adam", clip=None)
    ref = _reference_bf16(world, "adam", 4, round_sum=(strategy == "allreduce"))
    assert torch.equal(got["master"], ref), (got["master"] - ref).abs().max()


def _gather_worker(rank, world, port, out_dir):
    from k8s_amd.ops.optim import FusedAdam
    from k8s_amd.parallel.flat import ALIGN, ParamStore, init_normal
    from k8s_amd.parallel.ps import ShardedParameterService

    torch.set_num_threads(1)
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    store = ParamStore()
    [store.new("p%d" % i, s, init_normal(0.5)) for i, s in enumerate(SHAPES)]
    store.finalize("cpu", pad_to=world * ALIGN, seed=5)
    opt = FusedAdam(store, lr=0.01)
    svc = ShardedParameterService(store, opt, bucket_mb=0.002)
    for attr in opt.STATE:  # each rank's owned slices hold a recognisable pattern
        for lo, hi, off in opt.layout:
            getattr(opt, attr)[off:off + hi - lo] = torch.arange(lo, hi, dtype=torch.float32) * (
                1.0 if attr == "m1" else -1.0)
    full = svc.gather_state(dst=0)
    if rank == 0:
        n = store.total
        assert torch.equal(full["m1"], torch.arange(n, dtype=torch.float32))
        assert torch.equal(full["m2"], -torch.arange(n, dtype=torch.float32))
        assert not full["m1"].is_cuda  # host memory, never a full-size device copy
    else:
        assert full is None
    for attr in opt.STATE:
        getattr(opt, attr).zero_()
    src = {a: full[a] * 2 for a in full} if rank == 0 else None
    svc.scatter_state(src, src=0)
    for attr in opt.STATE:
        for lo, hi, off in opt.layout:
            want = torch.arange(lo, hi, dtype=torch.float32) * (2.0 if attr == "m1" else -2.0)
            assert torch.equal(getattr(opt, attr)[off:off + hi - lo], want)
    open(os.path.join(out_dir, "ok%d" % rank), "w").close()
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_state_gathers_to_one_rank_and_scatters_back():
    """checkpoints / PS snapshots gather the ZeRO-1 optimizer state to the chief only
    (bucket by bucket, into host memory), and a restore scatters each rank only its owned slices."""
    world = 4
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_gather_worker, args=(world, free_port(), d), nprocs=world)
        assert sorted(os.listdir(d)) == ["ok%d" % r for r in range(world)]


@pytest.mark.parametrize("world", [4, 8])
@pytest.mark.parametrize("comm", ["fp32", "bf16"])
def test_bf16_pull_bit_exact_against_fp32_pull(world, comm):
    """the ZeRO-1 bf16 pull (working copy all-gathered bucket by bucket, fp32 master kept
    sharded, fp32 all-gather only for the lowp=False parameters) ends bit-identical to the fp32-master pull after
    several Adam steps: master (after sync_master), bf16 copy and the gathered optimizer state; and before the sync
    the bf16 copy already equals bf16(master) everywhere."""
    a = _run(world, "ps", comm, "adam", steps=5, pull="lowp")
    b = _run(world, "ps", comm, "adam", steps=5, pull="fp32")
    assert a["stale_ok"]
    for k in ("master", "half", "exp_avg", "exp_avg_sq"):
        assert torch.equal(a[k], b[k]), k


def _check_worker(rank, world, port, out_dir, fault):
    from k8s_amd.ops.optim import FusedAdam
    from k8s_amd.parallel.ddp import GradReducer
    from k8s_amd.parallel.flat import ALIGN, ParamStore, init_normal
    from k8s_amd.parallel.ps import ShardedParameterService

    if fault:
        os.environ["K8S_AMD_FAULT_TRANSPORT"] = "1"
    torch.set_num_threads(1)
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    res = {}
    for strategy in ("allreduce", "ps"):
        for comm in ("fp32", "bf16"):
            store = ParamStore()
            for i, s in enumerate(SHAPES):
                store.new("p%d" % i, s, init_normal(0.5), lowp=(i % 3 != 2))
            store.finalize("cpu", pad_to=world * ALIGN, seed=5)
            dtype = torch.bfloat16 if comm == "bf16" else torch.float32
            before = store.grad.clone()
            if strategy == "ps":
                svc = ShardedParameterService(store, FusedAdam(store, lr=0.01), bucket_mb=0.002, comm_dtype=dtype,
                                              pull="lowp")
                r = svc.self_check()
                # the bf16 pull is issued in ascending offset order (first layers first)
                svc.step()
                offs = [svc.buckets[i].lo for i in svc.pull_order]
                r["pull_ascending"] = offs == sorted(offs)
                store.wait_pending()
            else:
                r = GradReducer(store, bucket_mb=0.002, comm_dtype=dtype).self_check()
                r["restored"] = torch.equal(before, store.grad)
            res["%s-%s" % (strategy, comm)] = r
    if rank == 0:
        torch.save(res, os.path.join(out_dir, "check.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("fault", [False, True])
def test_transport_self_check(fault):
    """the step-0 self-check of every gradient transport (all-reduce fp32/bf16, ZeRO-1
    push fp32/bf16) passes on a healthy 4-rank world, restores the gradient range it used, and fails every
    transport when the reduction is deliberately corrupted."""
    world = 4
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_check_worker, args=(world, free_port(), d, fault), nprocs=world)
        res = torch.load(os.path.join(d, "check.pt"), weights_only=True)
    assert sorted(res) == ["allreduce-bf16", "allreduce-fp32", "ps-bf16", "ps-fp32"]
    for name, r in res.items():
        assert r["world"] == world, name
        assert r["ok"] is (not fault), (name, r)
        if fault:
            assert r["max_err_over_tol"] > 10, (name, r)
        if name.startswith("ps"):
            assert r["pull_ascending"], name
        else:
            assert r["restored"], name
