"""BERT / Llama on the HIP kernels: bf16 GPU loss vs the fp32 CPU model with identical weights, and a few
optimizer steps that must reduce the loss."""
import pytest
import torch

from k8s_amd.models.registry import build
from k8s_amd.ops.optim import FusedAdam

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def no_aten_products():
    """every conv and linear product of these models runs on our kernels (no ATen
    fallback is counted), so the tests exercise the HIP path end to end."""
    from k8s_amd.ops import conv, gemm

    before = dict(conv.STATS)
    gemm.FALLBACKS.clear()
    yield
    aten = {k: conv.STATS[k] - before[k] for k in conv.STATS if k.startswith("aten_")}
    assert not any(aten.values()), aten
    assert gemm.FALLBACKS == {}, gemm.FALLBACKS


@pytest.mark.parametrize("name", ["bert_tiny", "llama_tiny"])
def test_loss_matches_cpu_fp32(cuda, name):
    g = build(name, cuda, batch=4, seed=3)
    c = build(name, "cpu", batch=4, seed=3)
    inputs = tuple(t.cpu() for t in g.batch(0))
    lc = c.loss(inputs).item()
    lg = g.loss(g.batch(0)).float().item()
    assert abs(lg - lc) < 3e-2 * max(1.0, abs(lc)), (lg, lc)


@pytest.mark.parametrize("name", ["bert_tiny", "llama_tiny", "resnet_tiny"])
def test_training_reduces_loss(cuda, name):
    w = build(name, cuda, batch=8, seed=1)
    opt = FusedAdam(w.store, lr=3e-3, weight_decay=0.0)
    losses = []
    for step in range(8):
        w.store.begin_step()
        loss = w.loss(w.batch(step))
        loss.backward()
        w.store.zero_unwritten()
        opt.step()
        losses.append(float(loss.float().item()))
    assert all(x == x for x in losses)
    assert losses[-1] < losses[0] * 0.9, losses
