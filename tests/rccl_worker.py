"""Worker for tests/test_rccl_gpu.py (not collected): a ONE-rank RCCL process group on the test box's GPU, with the
gradient transports force-enabled, so every collective they issue -- ``all_reduce``, ``all_to_all_single``,
``reduce_scatter_tensor``, ``all_gather_into_tensor`` -- runs as an RCCL kernel on gfx950 and the side-stream /
lazily-waited orderings (``Work.wait`` on a non-current stream, ``Param.weight``'s pull wait) are exercised on the
device. With one rank every reduction is the identity, so the results are exact: fp32 transport == the gradient,
bf16 transport == the gradient rounded to bf16 once, fp32 SGD at lr 1 == master - gradient. Prints one JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch.distributed as dist  # noqa: E402

from k8s_amd.ops.optim import FusedSGD  # noqa: E402
from k8s_amd.parallel import dist as kdist  # noqa: E402
from k8s_amd.parallel.ddp import GradReducer  # noqa: E402
from k8s_amd.parallel.flat import ParamStore, init_normal  # noqa: E402
from k8s_amd.parallel.ps import ShardedParameterService  # noqa: E402

SHAPES = [(4096, 1024), (1000,), (3, 3, 256, 256), (777,), (2048, 2048), (64,), (513, 129)]


def make_store(dev):
    st = ParamStore()
    for i, sh in enumerate(SHAPES):
        st.new("p%d" % i, sh, init_normal(0.02), decay=False, lowp=len(sh) > 1)
    return st.finalize(dev)


def backward_like(st, grads, busy):
    """Deposit the gradients in reverse order with GPU work in between (so the transports overlap real kernels)."""
    for p in reversed(st.params):
        busy.copy_(busy @ busy * 1e-3)
        st.deposit(p, grads[p.index])


def run_reducer(dev, comm, steps=10):
    st = make_store(dev)
    red = GradReducer(st, bucket_mb=4.0, enabled=True, comm_dtype=comm)
    check = red.self_check()
    busy = torch.randn(1024, 1024, device=dev)
    gen = torch.Generator(device=dev).manual_seed(7)
    worst, reserved = 0.0, []
    for _ in range(steps):
        grads = [torch.randn(p.shape, device=dev, generator=gen) for p in st.params]
        red.begin_step()
        backward_like(st, grads, busy)
        red.finish()
        want = torch.cat([(g.to(torch.bfloat16).float() if comm == torch.bfloat16 else g).reshape(-1)
                          for g in grads])
        got = torch.cat([p.grad.reshape(-1) for p in st.params])
        worst = max(worst, float((got - want).abs().max()))
        reserved.append(torch.cuda.memory_reserved(dev))
    return {"check": check, "max_abs_err": worst, "buckets": len(red.buckets), "reserved": reserved,
            "pool_bytes": red.pool.reserved_bytes}


def run_service(dev, comm, steps=10):
    st = make_store(dev)
    opt = FusedSGD(st, lr=1.0, momentum=0.0, weight_decay=0.0)
    svc = ShardedParameterService(st, opt, bucket_mb=4.0, comm_dtype=comm, enabled=True)
    check = svc.self_check()
    busy = torch.randn(1024, 1024, device=dev)
    gen = torch.Generator(device=dev).manual_seed(11)
    worst_m, worst_h, reserved = 0.0, 0.0, []
    for _ in range(steps):
        grads = [torch.randn(p.shape, device=dev, generator=gen) for p in st.params]
        before = st.master.clone()
        svc.begin_step()
        backward_like(st, grads, busy)
        svc.step()
        # the lazily-waited pull: read every weight through Param.weight (the forward's access path)
        halves = [p.weight.float().reshape(-1) for p in st.params if p.lowp]
        g = torch.zeros_like(before)
        for p in st.params:
            gp = grads[p.index].reshape(-1)
            g[p.offset:p.offset + p.numel] = gp.to(torch.bfloat16).float() if comm == torch.bfloat16 else gp
        want = before - g
        worst_m = max(worst_m, float((st.master - want).abs().max()))
        want_h = torch.cat([want[p.offset:p.offset + p.numel].to(torch.bfloat16).float()
                            for p in st.params if p.lowp])
        worst_h = max(worst_h, float((torch.cat(halves) - want_h).abs().max()))
        reserved.append(torch.cuda.memory_reserved(dev))
    return {"check": check, "max_abs_err_master": worst_m, "max_abs_err_half": worst_h, "pull": svc.pull,
            "sharded": svc.sharded, "reserved": reserved, "pool_bytes": svc.pool.reserved_bytes}


def main():
    info = kdist.init_process_group(backend="nccl", force=True)
    dev = torch.device("cuda", info.device_index)
    out = {"backend": str(dist.get_backend()), "world": dist.get_world_size()}
    for name, comm in (("fp32", torch.float32), ("bf16", torch.bfloat16)):
        out["reducer_" + name] = run_reducer(dev, comm)
        out["service_" + name] = run_service(dev, comm)
    torch.cuda.synchronize()
    print(json.dumps(out), flush=True)
    kdist.destroy()


if __name__ == "__main__":
    main()
