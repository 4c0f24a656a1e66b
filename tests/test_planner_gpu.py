"""Launch planners off the 256-CU grid.

Every grid-sizing rule (split-K cost model, stream-K tail, 256 vs 128 tile choice, persistent short-K grid, BN
reduction geometry, tiled weight-gradient grid, grid-stride caps) reads ``planner_cus()`` -- the device's
multiprocessor count unless overridden. In DP8 RCCL kernels occupy CUs next to backward, so a rank may plan for
fewer. Here the budget is forced to odd values and the products are checked against fp32 PyTorch references, and a
whole bottleneck block's forward/backward against the same block planned for the full chip.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _C():
    from k8s_amd.ops._ext import load

    return load()


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-6)).item()


@pytest.fixture
def budget_reset():
    yield
    _C().set_planner_cus(0)


def test_planner_reads_the_device_cu_count(cuda, budget_reset):
    C_ = _C()
    C_.set_planner_cus(0)
    assert C_.planner_cus() == torch.cuda.get_device_properties(cuda).multi_processor_count
    C_.set_planner_cus(77)
    assert C_.planner_cus() == 77
    C_.set_planner_cus(0)
    assert C_.planner_cus() == torch.cuda.get_device_properties(cuda).multi_processor_count


@pytest.mark.parametrize("cus", [96, 200])
def test_products_under_a_reduced_cu_budget(cuda, budget_reset, cus):
    C_ = _C()
    C_.set_planner_cus(cus)
    torch.manual_seed(cus)
    # 11 x 11 = 121 tiles of 256: at 96 CUs one full wave + a 25-tile stream-K tail (3-way K split), at 200 a
    # sub-wave grid that stays on the 128 x 128 kernel
    M = N = 2816
    K = 1536
    a = torch.randn(M, K, device=cuda).bfloat16()
    b = torch.randn(N, K, device=cuda).bfloat16()
    ref = a.float() @ b.float().t()
    for ak, bk in ((True, True), (False, False)):
        A = a if ak else a.t().contiguous()
        B = b if bk else b.t().contiguous()
        c = C_.gemm(A, ak, B, bk, None, True, None, 0, None, False, 1.0, 1)
        assert _rel(c, ref) < 1e-3, (ak, bk)
    # tall-K weight-gradient form with the split-K cost model choosing the splits (splits=0)
    g = torch.randn(50176, 256, device=cuda).bfloat16()
    x = torch.randn(50176, 512, device=cuda).bfloat16()
    out = torch.zeros(256, 512, device=cuda)
    C_.gemm(g, False, x, False, out, True, None, 0, None, True, 1.0, 0)
    assert _rel(out, g.float().t() @ x.float()) < 2e-3
    # short-K persistent kernel (1x1 conv forward with statistics), row count with a tail
    Mr, Kc, Nc = 300007, 64, 256
    xs = torch.randn(1, 1, Mr, Kc, device=cuda).bfloat16()
    ws = (torch.randn(Nc, 1, 1, Kc, device=cuda) * Kc ** -0.5).bfloat16()
    st = torch.zeros(C_.conv_stat_replicas, 2, Nc, device=cuda)
    y = C_.conv_fwd(xs, ws, 1, 0, 1, False, None, 0, st)
    yref = xs.reshape(Mr, Kc).float() @ ws.reshape(Nc, Kc).float().t()
    assert _rel(y.reshape(Mr, Nc), yref) < 1e-2
    torch.testing.assert_close(st.sum(0)[0], y.float().reshape(Mr, Nc).sum(0), rtol=2e-3, atol=5e-2)
    # staged-window 3x3 forward
    x3 = torch.randn(2, 56, 56, 64, device=cuda).bfloat16()
    w3 = (torch.randn(64, 3, 3, 64, device=cuda) / 24.0).bfloat16()
    y3 = C_.conv_fwd(x3, w3, 1, 1, 1, False, None, 0, None)
    r3 = F.conv2d(x3.float().permute(0, 3, 1, 2), w3.float().permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)
    assert _rel(y3, r3) < 1e-2


def _bottleneck_run(cuda, stride, downsample):
    from k8s_amd.models import resnet
    from k8s_amd.parallel.flat import ParamStore

    torch.manual_seed(9)
    store = ParamStore()
    blk = resnet.Bottleneck(store, "b", 256, 64, stride, downsample)
    store.finalize(cuda, seed=13)
    store.by_name["b.bn3.weight"].master.fill_(1.0)
    blk.to(cuda)
    x = torch.randn(8, 56, 56, 256, device=cuda).bfloat16().requires_grad_(True)
    store.begin_step()
    y = blk(x)
    y.float().square().mean().backward()
    return y.detach().float(), x.grad.float(), store.grad.clone()


@pytest.mark.parametrize("stride,down", [(1, False), (2, True)])
def test_bottleneck_planned_for_fewer_cus_matches_full_chip(cuda, budget_reset, stride, down):
    """BatchNorm geometry, split-K weight gradients, short-K and tiled kernels all re-planned for 120 CUs: the block's
    output, input gradient and every parameter gradient agree with the full-chip plan to fp32-summation order."""
    C_ = _C()
    C_.set_planner_cus(0)
    full = _bottleneck_run(cuda, stride, down)
    C_.set_planner_cus(120)
    few = _bottleneck_run(cuda, stride, down)
    assert _rel(few[0], full[0]) < 1e-3
    assert _rel(few[1], full[1]) < 5e-3
    assert _rel(few[2], full[2]) < 5e-3
