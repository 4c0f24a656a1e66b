"""End-to-end ResNet step on the GPU through the HIP kernels, checked against the CPU fp32 path."""
import pytest
import torch

from k8s_amd.models.resnet import resnet_tiny
from k8s_amd.ops import nn as K
from k8s_amd.ops.optim import FusedSGD
from k8s_amd.parallel.ddp import GradReducer
from k8s_amd.parallel.flat import ParamStore

pytestmark = pytest.mark.gpu


def _run(dev, dtype, steps=3):
    torch.manual_seed(0)
    store = ParamStore()
    m = resnet_tiny(store).finalize(dev)
    m.train()
    red = GradReducer(store)
    opt = FusedSGD(store, lr=0.05)
    g = torch.Generator().manual_seed(5)
    x = m.prepare_input(torch.randn(8, 32, 32, 3, generator=g)).to(dev, dtype).contiguous()
    y = torch.randint(0, 10, (8,), generator=g).to(dev)
    losses = []
    for _ in range(steps):
        red.begin_step()
        loss = K.cross_entropy(m(x), y)
        loss.backward()
        red.finish()
        opt.step()
        losses.append(float(loss.detach()))
    return losses, store


def test_resnet_tiny_gpu_matches_cpu(cuda):
    lg, sg = _run(cuda, torch.bfloat16)
    lc, sc = _run("cpu", torch.float32)
    assert all(abs(a - b) < 0.15 * max(1.0, abs(b)) for a, b in zip(lg, lc)), (lg, lc)
    assert lg[-1] < lg[0]
