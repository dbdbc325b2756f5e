"""Concurrent dgrad / wgrad schedules must produce exactly the gradients of the sequential one (same kernels,
same per-kernel reduction order): the opt-in weight-gradient side stream (ops/streams.py) eagerly, inside a
captured hipGraph and through the fused-MLP launch sequence, and the paired dgrad + wgrad GEMM launch
(pde::gemm_bf16_pair, the default) for every ResNet-50 / MLP pair configuration, also against fp32 PyTorch."""
import copy

import pytest
import torch

from pytorch_distributed_examples_amd.models.mlp import MLP
from pytorch_distributed_examples_amd.models.resnet import ResNet50, ResNetShard1
from pytorch_distributed_examples_amd.ops import functional as OF
from pytorch_distributed_examples_amd.ops import streams
from pytorch_distributed_examples_amd.ops.optim import FusedSGD

pytestmark = pytest.mark.gpu


def _grads(model, x, t, loss_fn, side: bool):
    for p in model.parameters():  # .grad must exist: the kernels accumulate straight into it
        p.grad = torch.zeros_like(p)
    old = streams.enabled()
    streams.set_enabled(side)
    try:
        loss_fn(model(x), t).backward()
    finally:
        streams.set_enabled(old)
    torch.cuda.synchronize()
    return [p.grad.clone() for p in model.parameters()]


def test_resnet_shard_side_stream_bitwise(gpu):
    torch.manual_seed(0)
    m = ResNetShard1().to(gpu)
    x = torch.randn(8, 3, 64, 64, device=gpu)
    t = torch.randn(8, 512, 8, 8, device=gpu)

    def loss_fn(out, tt):
        return OF.mse_loss(out.float().permute(0, 3, 1, 2)[:, :512], tt)

    g_one = _grads(m, x, t, loss_fn, side=False)
    g_two = _grads(m, x, t, loss_fn, side=True)
    for (n, _), a, b in zip(m.named_parameters(), g_one, g_two):
        assert torch.equal(a, b), n
    assert any(g.abs().sum() > 0 for g in g_two)


def test_mlp_side_stream_bitwise(gpu):
    torch.manual_seed(0)
    m = MLP(hidden_layers=5, features=1024).to(gpu)
    x = torch.randn(128, 1, 28, 28, device=gpu)
    y = torch.randint(0, 10, (128,), device=gpu)
    g_one = _grads(m, x, y, OF.cross_entropy, side=False)
    g_two = _grads(m, x, y, OF.cross_entropy, side=True)
    for (n, _), a, b in zip(m.named_parameters(), g_one, g_two):
        assert torch.equal(a, b), n


def test_fused_mlp_side_stream_bitwise(gpu):
    from pytorch_distributed_examples_amd.models.mlp_fused import FusedMLP

    torch.manual_seed(0)
    m = MLP(hidden_layers=5, features=1024).to(gpu)
    f = FusedMLP(m)
    x = torch.randn(128, 1, 28, 28, device=gpu)
    y = torch.randint(0, 10, (128,), device=gpu)
    out = []
    old = streams.enabled()
    for side in (False, True):
        streams.set_enabled(side)
        try:
            f.forward_backward(x, y)
        finally:
            streams.set_enabled(old)
        torch.cuda.synchronize()
        out.append([p.grad.clone() for p in m.parameters()])
    for a, b in zip(*out):
        assert torch.equal(a, b)


def test_resnet_graph_step_with_side_stream(gpu):
    """A captured training step (forward, backward with the default paired dgrad + wgrad launches and the
    deferred batched wgrad reduction, SGD) replays to the same weights as the same steps run eagerly.  (With
    PDE_WGRAD_STREAM=1 the same test covers the side-stream fork / join inside the capture: passed on MI355X
    while that was the default, r2k.)"""
    from pytorch_distributed_examples_amd.utils.graph import CapturedStep

    torch.manual_seed(0)
    ref = ResNet50().to(gpu)
    m = copy.deepcopy(ref)
    x = torch.randn(4, 3, 64, 64, device=gpu)
    t = torch.randn(4, 1000, device=gpu)

    def make_step(model, opt):
        def step(xx, tt):
            for p in model.parameters():
                if p.grad is not None:
                    p.grad.zero_()
            loss = OF.mse_loss(model(xx), tt)
            loss.backward()
            opt.step()
            return loss
        return step

    for p in list(ref.parameters()) + list(m.parameters()):
        p.grad = torch.zeros_like(p)
    opt_ref, opt = FusedSGD(ref.parameters(), lr=0.05), FusedSGD(m.parameters(), lr=0.05)
    step_ref = make_step(ref, opt_ref)
    with streams.disabled():
        for _ in range(3 + 4):  # CapturedStep warmup (3) + replays (4)
            step_ref(x, t)
    graph = CapturedStep(make_step(m, opt), (x, t), warmup=3).capture()
    for _ in range(4):
        graph(x, t)
    torch.cuda.synchronize()
    # capture itself runs no step (its kernels are recorded, not executed)
    for (n, a), b in zip(ref.named_parameters(), m.parameters()):
        assert torch.equal(a, b), n


# ---- dgrad + wgrad paired into one launch (pde::gemm_bf16_pair) ----------------------------------------------
# (N, H, W, Ci, Co, R, stride, pad): the ResNet-50 backward configurations at batch 32 / 128px -- every pair
# kind (3x3 gather dgrad, 1x1 dense / strided dgrad reading the forward copy transposed) with and without
# split-K on either side
PAIR_CONVS = [
    (32, 32, 32, 64, 64, 3, 1, 1),
    (32, 16, 16, 128, 128, 3, 1, 1),
    (32, 8, 8, 256, 256, 3, 1, 1),
    (32, 8, 8, 256, 256, 3, 2, 1),
    (32, 4, 4, 512, 512, 3, 1, 1),
    (32, 32, 32, 64, 256, 1, 1, 0),
    (32, 32, 32, 256, 64, 1, 1, 0),
    (32, 4, 4, 512, 2048, 1, 1, 0),
    (32, 16, 16, 512, 1024, 1, 2, 0),
    (8, 7, 7, 64, 64, 3, 1, 1),
]


@pytest.mark.parametrize("cfg", PAIR_CONVS, ids=[f"{c[1]}px_{c[3]}to{c[4]}_k{c[5]}s{c[6]}" for c in PAIR_CONVS])
def test_conv_dgrad_wgrad_pair_bitwise(gpu, cfg):
    n, h, w, ci, co, r, stride, pad = cfg
    C = OF._C()
    torch.manual_seed(0)
    ho, wo = (h + 2 * pad - r) // stride + 1, (w + 2 * pad - r) // stride + 1
    x = torch.randn(n, h, w, ci, device=gpu).to(torch.bfloat16)
    dy = torch.randn(n, ho, wo, co, device=gpu).to(torch.bfloat16)
    wt = torch.randn(co, ci, r, r, device=gpu) * 0.05
    if r == 1:
        wd, fwd_layout = C.cast_bf16(wt.contiguous()).view(co, ci), True
    else:
        wd, fwd_layout = C.conv_w_dgrad(wt.contiguous(), ci, co), False
    g_ref = torch.full_like(wt, 0.5)
    g_pair = g_ref.clone()
    dx_ref = C.conv_dgrad(dy, wd, h, w, r, r, stride, pad, None, fwd_layout, False)
    C.conv_wgrad(dy, x, r, r, stride, pad, co, ci, g_ref, True)
    with OF.gemm_pair():
        dx = C.conv_dgrad(dy, wd, h, w, r, r, stride, pad, None, fwd_layout, False)
        C.conv_wgrad(dy, x, r, r, stride, pad, co, ci, g_pair, True)
    torch.cuda.synchronize()
    assert torch.equal(dx, dx_ref)
    assert torch.equal(g_pair, g_ref)
    # and against fp32 PyTorch
    xf, dyf = x.float().permute(0, 3, 1, 2), dy.float().permute(0, 3, 1, 2)
    wq = wd.float().view(co, ci, 1, 1) if r == 1 else wt.to(torch.bfloat16).float()
    dx32 = torch.nn.grad.conv2d_input(xf.shape, wq, dyf, stride=stride, padding=pad)
    dw32 = torch.nn.grad.conv2d_weight(xf, wt.shape, dyf, stride=stride, padding=pad)
    err_x = ((dx.float().permute(0, 3, 1, 2) - dx32).norm() / dx32.norm()).item()
    err_w = ((g_pair - 0.5 - dw32).norm() / dw32.norm()).item()
    assert err_x < 1e-2 and err_w < 1e-3, (err_x, err_w)


@pytest.mark.parametrize("batch", [128, 37])
def test_linear_dgrad_wgrad_pair_bitwise(gpu, batch):
    C = OF._C()
    torch.manual_seed(0)
    k, nout = 1024, 1024
    dy = torch.randn(batch, nout, device=gpu).to(torch.bfloat16)
    x_ext = torch.zeros(batch, k + 8, device=gpu, dtype=torch.bfloat16)
    x_ext[:, :k] = torch.randn(batch, k, device=gpu).to(torch.bfloat16)
    x_ext[:, k] = 1.0
    aux = torch.relu(torch.randn(batch, k + 8, device=gpu)).to(torch.bfloat16)
    w = (torch.randn(nout, k, device=gpu) * 0.03).to(torch.bfloat16)
    outs = []
    for paired in (False, True):
        dx = torch.empty(batch, k + 8, device=gpu, dtype=torch.bfloat16)
        gw = torch.zeros(nout, k, device=gpu)
        gb = torch.zeros(nout, device=gpu)
        if paired:
            with OF.gemm_pair():
                C.linear_dgrad_out(dy, w, aux[:, :k], dx[:, :k])
                C.linear_wgrad_bias(dy, x_ext[:, :k + 1], gw, gb, False)
        else:
            C.linear_dgrad_out(dy, w, aux[:, :k], dx[:, :k])
            C.linear_wgrad_bias(dy, x_ext[:, :k + 1], gw, gb, False)
        torch.cuda.synchronize()
        outs.append((dx[:, :k].clone(), gw, gb))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    ref_gw = dy.float().t() @ x_ext[:, :k].float()
    assert ((outs[1][1] - ref_gw).norm() / ref_gw.norm()).item() < 1e-3
    assert torch.allclose(outs[1][2], dy.float().sum(0), rtol=1e-3, atol=1e-2)


# ---- deferred, batched weight-gradient reductions (ops/streams.py flush_deferred) ------------------------------
def _with_defer(flag, fn):
    old = streams._DEFER_ENABLED[0]
    streams._DEFER_ENABLED[0] = flag
    try:
        return fn()
    finally:
        streams._DEFER_ENABLED[0] = old


def test_deferred_wgrad_reduce_bitwise_resnet(gpu):
    """ResNet-50 (both shards, batch 32 at 64px: split-K weight gradients in every stage) -- gradients after
    backward() with the per-step batched reduction equal the per-layer reductions bit for bit, and nothing is
    left pending after backward returns."""
    torch.manual_seed(0)
    m = ResNet50().to(gpu)
    x = torch.randn(32, 3, 64, 64, device=gpu)
    t = torch.randn(32, 1000, device=gpu)
    g_now = _with_defer(False, lambda: _grads(m, x, t, OF.mse_loss, side=False))
    g_def = _with_defer(True, lambda: _grads(m, x, t, OF.mse_loss, side=False))
    assert OF._C().gemm_deferred_count() == 0
    for (n, _), a, b in zip(m.named_parameters(), g_now, g_def):
        assert torch.equal(a, b), n


def test_deferred_wgrad_reduce_bitwise_fused_mlp(gpu):
    from pytorch_distributed_examples_amd.models.mlp_fused import FusedMLP

    torch.manual_seed(0)
    m = MLP(hidden_layers=5, features=1024).to(gpu)
    f = FusedMLP(m)
    x = torch.randn(128, 1, 28, 28, device=gpu)
    y = torch.randint(0, 10, (128,), device=gpu)
    out = []
    for flag in (False, True):
        _with_defer(flag, lambda: f.forward_backward(x, y))
        torch.cuda.synchronize()
        out.append([p.grad.clone() for p in m.parameters()])
    assert OF._C().gemm_deferred_count() == 0
    for a, b in zip(*out):
        assert torch.equal(a, b)
