"""CPU tier: the model/store/optimizer/reducer stack trains (fp32 reference kernels)."""
import torch

from k8s_amd.models.resnet import resnet50, resnet_tiny
from k8s_amd.ops import nn as K
from k8s_amd.ops.optim import FusedAdam, FusedSGD
from k8s_amd.parallel.ddp import GradReducer
from k8s_amd.parallel.flat import ParamStore


def test_resnet50_param_count():
    s = ParamStore()
    resnet50(s)
    # torchvision resnet50 = 25,557,032; our stem reads 8 (zero-padded) input channels: +64*7*7*5
    assert s.num_parameters() == 25_557_032 + 64 * 7 * 7 * 5


def _train(opt_cls, steps=6, **kw):
    torch.manual_seed(0)
    store = ParamStore()
    m = resnet_tiny(store).finalize("cpu")
    red = GradReducer(store)
    opt = opt_cls(store, **kw)
    x = m.prepare_input(torch.randn(4, 32, 32, 3))
    y = torch.randint(0, 10, (4,))
    out = []
    for _ in range(steps):
        red.begin_step()
        loss = K.cross_entropy(m(x), y)
        loss.backward()
        red.finish()
        opt.step()
        out.append(float(loss.detach()))
    return out


def test_tiny_resnet_sgd_converges():
    l = _train(FusedSGD, lr=0.05)
    assert l[-1] < 0.5 * l[0]


def test_tiny_resnet_adam_converges():
    l = _train(FusedAdam, lr=3e-3, weight_decay=0.0)
    assert l[-1] < 0.5 * l[0]
