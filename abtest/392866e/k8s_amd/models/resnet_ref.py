"""Plain-PyTorch (NCHW, fp32, torch.nn.functional) functional twin of ``models.resnet`` for tests:
same weights (read from the flat store), same architecture, autograd for the gradients. Used to check the
hand-written NHWC/BN/conv/residual-fusion path end to end."""
from __future__ import annotations

from typing import Dict

import torch
import torch.nn.functional as F


def _conv(x, w_krsc, stride, pad):
    return F.conv2d(x, w_krsc.permute(0, 3, 1, 2), None, stride, pad)


def _bn(x, p, name, relu=True, res=None, eps=1e-5):
    y = F.batch_norm(x, None, None, p[name + ".weight"], p[name + ".bias"], training=True, eps=eps)
    if res is not None:
        y = y + res
    return torch.relu(y) if relu else y


def forward(model, params: Dict[str, torch.Tensor], images_nchw: torch.Tensor) -> torch.Tensor:
    """Logits of ``model`` (a models.resnet.ResNet) evaluated with plain ops on ``params`` (name -> fp32)."""
    x = _bn(_conv(images_nchw, params["conv1.weight"], 2, 3), params, "bn1")
    x = F.max_pool2d(x, 3, 2, 1)
    for b in model.blocks:
        name = b.conv1.w.name[:-len(".conv1.weight")]
        idn = x
        y = _bn(_conv(x, params[name + ".conv1.weight"], 1, 0), params, name + ".bn1")
        y = _bn(_conv(y, params[name + ".conv2.weight"], b.conv2.stride, 1), params, name + ".bn2")
        if b.down is not None:
            idn = _bn(_conv(x, params[name + ".downsample.0.weight"], b.down.stride, 0), params,
                      name + ".downsample.1", relu=False)
        x = _bn(_conv(y, params[name + ".conv3.weight"], 1, 0), params, name + ".bn3", res=idn)
    x = x.mean(dim=(2, 3))
    return F.linear(x, params["fc.weight"], params["fc.bias"])


def reference_grads(model, store, images_nhwc, labels, autocast_bf16=False):
    """(loss, {name: grad}) of the plain-op twin at the store's current fp32 master weights
    (``autocast_bf16``: the stock mixed-precision run of the same twin, to size bf16 noise)."""
    params = {p.name: p.master.detach().float().clone().requires_grad_(True) for p in store.params}
    x = images_nhwc.float().permute(0, 3, 1, 2)
    with torch.autocast(x.device.type, dtype=torch.bfloat16, enabled=autocast_bf16):
        loss = F.cross_entropy(forward(model, params, x).float(), labels)
    loss.backward()
    return loss.detach(), {k: v.grad for k, v in params.items()}
