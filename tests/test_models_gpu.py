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


def test_bert_full_vocab_decoder_matches_cpu_fp32(cuda):
    """BERT's tied MLM decoder at the full 30,522-word vocabulary -- padded to 30,720 columns so the logits, their
    data gradient and the tied table's gradient run on the 4-wave GEMM's 256-column tiles -- against the fp32 CPU
    model with identical weights: the loss (the padded logits masked out) and the decoder bias gradient."""
    import dataclasses

    from k8s_amd.models import bert as M
    from k8s_amd.parallel.flat import ParamStore

    cfg = dataclasses.replace(M.BERT_TINY, vocab_size=30522, hidden=256, intermediate=1024, heads=4, layers=1,
                              max_position=128, max_predictions=20)
    assert cfg.padded_vocab == 30720
    out = {}
    batch = None
    for dev, dt in ((cuda, torch.bfloat16), (torch.device("cpu"), torch.float32)):
        store = ParamStore()
        model = M.BertForPreTraining(store, cfg).finalize(dev, seed=5)
        if batch is None:
            gen = torch.Generator(device=dev)
            gen.manual_seed(7)
            batch = M.synthetic_batch(cfg, 64, 128, dev, generator=gen)  # 1,280 masked rows: 5 x 120 tiles
        b = tuple(t.to(dev) for t in batch)
        store.begin_step()
        loss = model(*b, dtype=dt)[0]
        loss.backward()
        store.zero_unwritten()
        out[dev.type] = (loss.float().item(), model.dec_b.grad.float().cpu().clone())
    lg, gg = out["cuda"]
    lc, gc = out["cpu"]
    assert abs(lg - lc) < 3e-2 * max(1.0, abs(lc)), (lg, lc)
    assert gg[30522:].abs().max().item() == 0.0  # padded logits carry no gradient
    err = ((gg - gc).norm() / gc.norm()).item()
    assert err < 5e-2, err
