"""Worker for tests/test_dist_gpu.py (not collected): DP training of resnet_tiny on the GPU kernels with the
bucketed GradReducer, then every rank's fp32 master weights and momentum are compared with rank 0's."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from k8s_amd.models.resnet import resnet_tiny  # noqa: E402
from k8s_amd.ops import nn as K  # noqa: E402
from k8s_amd.ops.optim import FusedSGD  # noqa: E402
from k8s_amd.parallel import dist as kdist  # noqa: E402
from k8s_amd.parallel.ddp import GradReducer  # noqa: E402
from k8s_amd.parallel.flat import ParamStore  # noqa: E402


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "allreduce-fp32"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    info = kdist.init_process_group()
    gpu = torch.cuda.is_available()
    dev = torch.device("cuda", info.device_index) if gpu else torch.device("cpu")  # CPU: a dry run of this script
    store = ParamStore()
    model = resnet_tiny(store).finalize(dev, pad_to=64 * info.world_size)
    torch.distributed.broadcast(store.master, 0)
    store.refresh_lowp()
    opt = FusedSGD(store, lr=0.05, momentum=0.9, weight_decay=1e-4)
    if mode.startswith("zero"):  # ZeRO-1 sharded service (reduce-scatter / all-to-all push, owner update, pull)
        from k8s_amd.parallel.ps import ShardedParameterService

        # "zero-fp32pull-*": the fp32-master pull; otherwise the GPU default, the bf16 working-copy pull
        svc = ShardedParameterService(store, opt, bucket_mb=0.01,
                                      comm_dtype=torch.bfloat16 if mode.endswith("bf16") else torch.float32,
                                      pull="fp32" if "fp32pull" in mode else "auto")
        begin, finish = svc.begin_step, svc.step
    else:  # many buckets: every hook / overlap path runs
        red = GradReducer(store, bucket_mb=0.01,
                          comm_dtype=torch.bfloat16 if mode.endswith("bf16") else torch.float32)
        begin = red.begin_step

        def finish():
            red.finish()
            opt.step(grad_scale=red.grad_scale)
    g = torch.Generator(device="cpu").manual_seed(100 + info.rank)  # different data per rank
    reserved = []  # caching-allocator reservation after each step: the bf16 transports must not grow it
    for _ in range(steps):
        x = torch.randn(8, 32, 32, 3, generator=g).to(dev, torch.bfloat16 if gpu else torch.float32)
        y = torch.randint(0, 10, (8,), generator=g).to(dev)
        begin()
        loss = K.cross_entropy(model(model.prepare_input(x).contiguous()), y)
        loss.backward()
        finish()
        reserved.append(torch.cuda.memory_reserved(dev) if gpu else 0)
    pull = "none"
    if mode.startswith("zero"):
        pull = svc.pull
        svc.sync_master()  # the bf16 pull keeps only the owned fp32 master slices current
    if gpu:
        torch.cuda.synchronize()
    # the sharded optimizer keeps different (owned) state slices per rank: compare the weights only
    state = (store.master if mode.startswith("zero") else torch.cat([store.master, opt.mom])).cpu()
    ref = state.clone()
    torch.distributed.broadcast(ref, 0)
    same = torch.tensor([int(torch.equal(state, ref))])
    torch.distributed.all_reduce(same, op=torch.distributed.ReduceOp.MIN)
    if info.rank == 0:
        print("{\"replicas_identical\": %d, \"world\": %d, \"loss\": %.5f, \"pull\": \"%s\", \"wsum\": %r, "
              "\"reserved\": %s}"
              % (int(same), info.world_size, float(loss.detach()), pull, float(store.master.double().sum()),
                 reserved), flush=True)
    kdist.destroy()


if __name__ == "__main__":
    main()
