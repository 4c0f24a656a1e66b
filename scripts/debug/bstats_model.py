"""Debug: per-parameter gradient difference between BN_BSTATS on / off on a small ResNet (GPU)."""
import sys

import torch

from k8s_amd.models.resnet import ResNet
from k8s_amd.ops import conv as kc
from k8s_amd.ops import nn as K
from k8s_amd.parallel.flat import ParamStore

cuda = torch.device("cuda")
layers = tuple(int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "3,3,2,1").split(","))
size = int(sys.argv[2]) if len(sys.argv) > 2 else 224
mode = sys.argv[3] if len(sys.argv) > 3 else "all"
batch = int(sys.argv[4]) if len(sys.argv) > 4 else 4


def run(on):
    K.BN_BSTATS = on
    torch.manual_seed(0)
    store = ParamStore()
    m = ResNet(store, layers, 10, width=64).finalize(cuda, seed=3)
    with torch.no_grad():
        gen = torch.Generator(device="cpu").manual_seed(11)
        for p in store.params:
            if "bn" in p.name or "downsample.1" in p.name:
                p.master.copy_((torch.rand(p.shape, generator=gen) * 0.8 + 0.6 if p.name.endswith("weight")
                                else torch.randn(p.shape, generator=gen) * 0.1).to(cuda))
    store.refresh_lowp()
    m.train()
    images = torch.randn(batch, size, size, 3, generator=torch.Generator(device="cpu").manual_seed(1)).to(cuda)
    x = m.prepare_input(images.bfloat16())
    y = torch.arange(batch, device=cuda) % 10
    n0 = kc.STATS["bn_bstats"]
    store.begin_step()
    loss = K.cross_entropy(m(x), y)
    loss.backward()
    store.zero_unwritten()
    torch.cuda.synchronize()
    return loss.item(), {p.name: p.grad.float().clone() for p in store.params}, kc.STATS["bn_bstats"] - n0


if mode == "conv3x3only":
    import k8s_amd.ops.conv as c
    orig = c._dgrad_hip
l1, g1, n1 = run(mode != "offoff")
l0, g0, n0 = run(False)
print("loss", l1, l0, "fused calls", n1, n0)
for name, r in g0.items():
    err = (g1[name] - r).norm().item() / (r.norm().item() + 1e-6)
    print("%-32s %.4f" % (name, err))
