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


def test_resnet_tiny_gradients_match_plain_pytorch():
    """Loss and every parameter gradient of the NHWC op path (fused BN+ReLU+residual, the residual-gradient
    link into conv1's dgrad, flat-store deposits) against a plain torch.nn.functional twin."""
    from k8s_amd.models.resnet_ref import reference_grads
    from k8s_amd.ops import nn as K

    from k8s_amd.models.resnet import ResNet

    torch.manual_seed(0)
    store = ParamStore()
    m = ResNet(store, (2, 2, 1, 1), 10, width=8).finalize("cpu", seed=3)  # identity blocks in stages 1-2
    m.train()
    x = m.prepare_input(torch.randn(4, 32, 32, 3))
    y = torch.randint(0, 10, (4,))
    store.begin_step()
    loss = K.cross_entropy(m(x), y)
    loss.backward()
    store.zero_unwritten()
    ref_loss, ref = reference_grads(m, store, x, y)
    assert abs(loss.item() - ref_loss.item()) < 1e-4
    for p in store.params:
        g, r = p.grad.float(), ref[p.name]
        err = (g - r).abs().max().item()
        assert err <= 1e-3 * max(1.0, r.abs().max().item()), (p.name, err)


def test_strided_dgrad_parity_taps():
    """Output-parity decomposition of a stride-s data gradient (ops/conv.py): the taps of every parity,
    emulated with stride-1 correlations on CPU, reproduce ATen's convolution_backward exactly."""
    import torch.nn.functional as F

    from k8s_amd.ops import conv

    torch.manual_seed(0)
    for (N, H, C, K, R, s, p) in [(2, 8, 16, 64, 3, 2, 1), (2, 9, 16, 64, 3, 2, 1), (2, 8, 16, 64, 1, 2, 0),
                                  (1, 7, 8, 64, 7, 2, 3)]:
        x, w = torch.randn(N, H, H, C), torch.randn(K, R, R, C)
        Ho = (H + 2 * p - R) // s + 1
        gy = torch.randn(N, Ho, Ho, K)
        assert conv.strided_dgrad_ok(gy, w, s, p)
        dx = torch.empty(N, H, H, C)
        for a in range(s):
            tr = conv._parity_taps(R, a, p, s)
            for b in range(s):
                ts = conv._parity_taps(R, b, p, s)
                if not tr or not ts:
                    dx[:, a::s, b::s] = 0
                    continue
                wr = torch.stack([w[:, r] for _, r in tr], dim=1)
                wsub = torch.stack([wr[:, :, q] for _, q in ts], dim=2)  # [K, Tr, Ts, C]
                Hs, Ws = (H - a + s - 1) // s, (H - b + s - 1) // s
                lo = -tr[0][0]
                xin = F.pad(gy.permute(0, 3, 1, 2), (lo, Ws - (Ho + lo - len(ts) + 1), lo, Hs - (Ho + lo - len(tr) + 1)))
                dx[:, a::s, b::s] = F.conv2d(xin, wsub.permute(3, 0, 1, 2)).permute(0, 2, 3, 1)
        ref = torch.ops.aten.convolution_backward(gy.permute(0, 3, 1, 2), x.permute(0, 3, 1, 2),
                                                  w.permute(0, 3, 1, 2), None, [s, s], [p, p], [1, 1], False,
                                                  [0, 0], 1, [True, False, False])[0].permute(0, 2, 3, 1)
        assert (dx - ref).abs().max() < 1e-3


def test_shared_grad_link_sums_both_readers_in_either_order():
    """A downsample block's x feeds conv1 and the strided downsample conv through one shared GradLink: the
    first backward hands its dx over, the second adds it in its dgrad. Whichever order autograd picks, x.grad
    must equal the plain sum of both convolutions' input gradients."""
    import torch.nn.functional as F

    from k8s_amd.parallel.flat import init_kaiming_normal

    for down_first in (False, True):
        torch.manual_seed(3)
        store = ParamStore()
        pa = store.new("a.weight", (16, 1, 1, 8), init_kaiming_normal(8))
        pb = store.new("b.weight", (16, 1, 1, 8), init_kaiming_normal(8))
        store.finalize("cpu")
        x = torch.randn(2, 8, 8, 8, requires_grad=True)
        link = K.GradLink(shared=True)
        store.begin_step()
        if down_first:  # created later in forward -> runs earlier in backward
            ya = K.conv2d_nhwc(x, pa, 1, 0, grad_link=link)
            yb = K.conv2d_nhwc(x, pb, 2, 0, grad_link=link)
        else:
            yb = K.conv2d_nhwc(x, pb, 2, 0, grad_link=link)
            ya = K.conv2d_nhwc(x, pa, 1, 0, grad_link=link)
        ga, gb = torch.randn_like(ya), torch.randn_like(yb)
        ((ya * ga).sum() + (yb * gb).sum()).backward()
        assert link.grad is None  # consumed by the second reader
        xr = x.detach().permute(0, 3, 1, 2).requires_grad_(True)
        wa = pa.master.view(16, 1, 1, 8).permute(0, 3, 1, 2)
        wb = pb.master.view(16, 1, 1, 8).permute(0, 3, 1, 2)
        ((F.conv2d(xr, wa) * ga.permute(0, 3, 1, 2)).sum()
         + (F.conv2d(xr, wb, stride=2) * gb.permute(0, 3, 1, 2)).sum()).backward()
        torch.testing.assert_close(x.grad, xr.grad.permute(0, 2, 3, 1), rtol=1e-4, atol=1e-4)
