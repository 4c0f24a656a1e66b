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


def test_resnet_gradients_match_plain_pytorch_gpu(cuda):
    """bf16 NHWC kernel path (implicit-GEMM convs with fused BN statistics, fused BN+ReLU+residual, residual
    gradient accumulated in conv1's dgrad epilogue) vs an fp32 torch.nn.functional twin on the same weights."""
    from k8s_amd.models.resnet import ResNet
    from k8s_amd.models.resnet_ref import reference_grads
    from k8s_amd.ops import nn as K
    from k8s_amd.parallel.flat import ParamStore

    torch.manual_seed(0)
    store = ParamStore()
    m = ResNet(store, (2, 2, 1, 1), 10, width=64).finalize(cuda, seed=3)
    m.train()
    x = m.prepare_input(torch.randn(8, 64, 64, 3, device=cuda).bfloat16())
    y = torch.randint(0, 10, (8,), device=cuda)
    store.begin_step()
    loss = K.cross_entropy(m(x), y)
    loss.backward()
    store.zero_unwritten()
    ref_loss, ref = reference_grads(m, store, x, y)
    _, stock = reference_grads(m, store, x, y, autocast_bf16=True)  # stock bf16 autocast: the noise floor
    assert abs(loss.float().item() - ref_loss.item()) < 3e-2 * max(1.0, abs(ref_loss.item()))
    bad = []
    for p in store.params:
        r = ref[p.name].float()
        err = (p.grad.float() - r).norm().item() / (r.norm().item() + 1e-6)
        floor = (stock[p.name].float() - r).norm().item() / (r.norm().item() + 1e-6)
        if err > 2.0 * floor + 0.03:
            bad.append((p.name, round(err, 3), round(floor, 3)))
    assert not bad, bad
