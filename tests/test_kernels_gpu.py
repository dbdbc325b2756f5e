"""Numerics of every gfx950 kernel against a plain PyTorch fp32 reference of the same op.

Inputs are random and asymmetric (cdna_hip_programming.md §3: an asymmetric operand catches swapped
C/D layouts); tolerances are set for bf16 operands with fp32 accumulation.
"""
import pytest
import torch
import torch.nn.functional as F

from pytorch_distributed_examples_amd.ops import functional as OF

pytestmark = pytest.mark.gpu


def bf(x):
    return x.to(torch.bfloat16).float()


def rel_err(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("M,K,N", [(128, 784, 1024), (128, 1024, 10), (1000, 320, 50), (37, 50, 10),
                                   (2048, 2048, 1000), (8, 64, 128)])
def test_linear_fwd_bwd(gpu, M, K, N):
    C = OF._C()
    torch.manual_seed(0)
    x = torch.randn(M, K, device=gpu)
    w = torch.randn(N, K, device=gpu) * 0.05
    b = torch.randn(N, device=gpu)
    xb, wb = x.bfloat16(), w.bfloat16()
    y = C.linear_fwd(xb, wb, b, True, True)
    ref = torch.relu(bf(x) @ bf(w).t() + b)
    assert rel_err(y, ref) < 1e-2
    dy = torch.randn(M, N, device=gpu).bfloat16()
    dx = C.linear_dgrad(dy, wb, None)
    assert rel_err(dx, dy.float() @ bf(w)) < 1e-2
    aux = torch.randn(M, K, device=gpu).bfloat16()
    dxm = C.linear_dgrad(dy, wb, aux)
    assert rel_err(dxm, (dy.float() @ bf(w)) * (aux.float() > 0)) < 1e-2
    dw = C.linear_wgrad(dy, xb)
    assert rel_err(dw, dy.float().t() @ bf(x)) < 1e-2


@pytest.mark.parametrize("M,K,N", [(128, 1024, 1024), (200, 4096, 96), (72, 2056, 40), (1000, 320, 56)])
def test_skinny_gemm_paths(gpu, M, K, N):
    """Few output tiles over a long K: the in-block wave split-K kernel (gemm.hip skinny_tile) -- forward
    (K-contiguous weight, bias + ReLU epilogue), dgrad (row-contiguous weight through the transposing LDS
    image, ReLU-mask epilogue), several K batches and ragged M / N edges; bitwise deterministic."""
    C = OF._C()
    torch.manual_seed(1)
    x = torch.randn(M, K, device=gpu).bfloat16()
    w = (torch.randn(N, K, device=gpu) * 0.05).bfloat16()
    b = torch.randn(N, device=gpu)
    y = C.linear_fwd(x, w, b, True, False)
    assert rel_err(y, torch.relu(x.float() @ w.float().t() + b)) < 1e-2
    assert torch.equal(y, C.linear_fwd(x, w, b, True, False))
    wt = (torch.randn(K, N, device=gpu) * 0.05).bfloat16()  # dgrad-shaped: dx[M, N] = dy2[M, K] @ wt[K, N]
    dy2 = torch.randn(M, K, device=gpu).bfloat16()
    aux = torch.randn(M, N, device=gpu).bfloat16()
    dx = C.linear_dgrad(dy2, wt, aux)
    assert rel_err(dx, (dy2.float() @ wt.float()) * (aux.float() > 0)) < 1e-2


def test_linear_identity_asymmetric(gpu):
    """A = I with an asymmetric B catches a transposed C write."""
    C = OF._C()
    n = 64
    eye = torch.eye(n, device=gpu).bfloat16()
    B = (torch.arange(n * n, device=gpu).reshape(n, n) % 61).float().bfloat16()
    y = C.linear_fwd(eye, B, None, False, True)
    assert torch.equal(y, B.float().t())


# Every unique conv of the ResNet-50 shards at 128x128 (model_parallel_ResNet50.py:94-130):
# (Cin, Cout, k, stride, pad, H_in), micro-batch 4; plus the two MNIST convs (mnist_horovod.py:9-25).
RESNET_CONVS = [
    # shard 1: stem + layer1 + layer2
    (3, 64, 7, 2, 3, 128), (64, 64, 1, 1, 0, 32), (64, 64, 3, 1, 1, 32), (64, 256, 1, 1, 0, 32),
    (256, 64, 1, 1, 0, 32), (256, 128, 1, 1, 0, 32), (128, 128, 3, 2, 1, 32), (256, 512, 1, 2, 0, 32),
    (128, 512, 1, 1, 0, 16), (128, 128, 3, 1, 1, 16), (512, 128, 1, 1, 0, 16),
    # shard 2: layer3 + layer4
    (512, 256, 1, 1, 0, 16), (256, 256, 3, 2, 1, 16), (512, 1024, 1, 2, 0, 16), (256, 1024, 1, 1, 0, 8),
    (256, 256, 3, 1, 1, 8), (1024, 256, 1, 1, 0, 8), (1024, 512, 1, 1, 0, 8), (512, 512, 3, 2, 1, 8),
    (1024, 2048, 1, 2, 0, 8), (512, 2048, 1, 1, 0, 4), (512, 512, 3, 1, 1, 4), (2048, 512, 1, 1, 0, 4),
]
CONV_CFGS = [(4, ci, h, co, k, s, p) for ci, co, k, s, p, h in RESNET_CONVS] + [
    # N, Cin, H, Cout, k, stride, pad
    (8, 1, 28, 10, 5, 1, 0),      # MNIST conv1
    (8, 10, 12, 20, 5, 1, 0),     # MNIST conv2
]
assert len(CONV_CFGS) == 25


@pytest.mark.parametrize("cfg", CONV_CFGS)
def test_conv_fwd_bwd(gpu, cfg):
    n, ci, h, co, k, s, p = cfg
    torch.manual_seed(1)
    x = torch.randn(n, ci, h, h, device=gpu)
    w = (torch.randn(co, ci, k, k, device=gpu) * (1.0 / (ci * k * k) ** 0.5)).requires_grad_()
    b = torch.randn(co, device=gpu).requires_grad_()
    xr = bf(x).requires_grad_()
    yr = F.conv2d(xr, bf(w.detach()).requires_grad_(), b, stride=s, padding=p)
    # native
    xn = OF.to_native_image(x).requires_grad_()
    yn = OF.conv2d(xn, w, b, s, p)
    y_nchw = yn[..., :co].permute(0, 3, 1, 2).float()
    assert rel_err(y_nchw, yr) < 1.5e-2
    g = torch.randn_like(yr)
    gn = torch.zeros_like(yn, dtype=torch.float32)
    gn[..., :co] = g.permute(0, 2, 3, 1)
    (yn.float() * gn).sum().backward()
    wr = bf(w.detach()).requires_grad_()
    xr2 = bf(x).requires_grad_()
    F.conv2d(xr2, wr, b.detach(), stride=s, padding=p).backward(g)
    assert rel_err(w.grad, wr.grad) < 2e-2
    assert rel_err(b.grad, g.sum((0, 2, 3))) < 1e-2
    dx = xn.grad[..., :ci].permute(0, 3, 1, 2)
    assert rel_err(dx, xr2.grad) < 2e-2
    if xn.shape[-1] > ci:
        assert xn.grad[..., ci:].abs().max().item() == 0.0


@pytest.mark.parametrize("M,N", [(128, 1024), (37, 16), (1024, 264), (1025, 64), (5000, 1000), (64, 10)])
def test_colsum(gpu, M, N):
    """Bias-gradient column sums (single-launch short path for M <= 1024, two-level beyond, scalar for
    N % 8 != 0), written and accumulated, against an fp32 torch sum."""
    C = OF._C()
    torch.manual_seed(5)
    x = torch.randn(M, N, device=gpu).bfloat16()
    ref = x.float().sum(0)
    out = C.colsum(x, N, torch.zeros(N, device=gpu), False)
    assert rel_err(out, ref) < 1e-4
    base = torch.randn(N, device=gpu)
    acc = C.colsum(x, N, base.clone(), True)
    assert rel_err(acc, base + ref) < 1e-4


# shapes: one 64-channel slice; C < 64 (partial slice, groups not dividing 256); C % 64 != 0 (ragged
# last slice, several slices); many rows (256 row chunks per slice -> widest last-block combine); odd row
# counts per chunk (P = 1000, 3600).
@pytest.mark.parametrize("relu,res,n,c,h", [(False, False, 8, 64, 16), (True, False, 8, 64, 16),
                                            (True, True, 8, 64, 16), (True, False, 4, 24, 10),
                                            (False, True, 2, 200, 9), (True, True, 32, 64, 64),
                                            (False, False, 2, 2048, 4), (True, True, 10, 96, 10),
                                            (True, True, 16, 64, 32), (False, True, 4, 200, 30)])
def test_batchnorm(gpu, relu, res, n, c, h):
    torch.manual_seed(2)
    x = torch.randn(n, c, h, h, device=gpu) * 3 + 1
    gamma = (torch.rand(c, device=gpu) + 0.5).requires_grad_()
    beta = torch.randn(c, device=gpu).requires_grad_()
    r = torch.randn(n, c, h, h, device=gpu) if res else None
    rm, rv = torch.zeros(c, device=gpu), torch.ones(c, device=gpu)
    xn = bf(x).permute(0, 2, 3, 1).contiguous().bfloat16().requires_grad_()
    rn = bf(r).permute(0, 2, 3, 1).contiguous().bfloat16().requires_grad_() if res else None
    y = OF.batch_norm(xn, gamma, beta, rm, rv, True, 0.1, 1e-5, rn, relu)
    # reference
    xr = bf(x).requires_grad_()
    g2, b2 = gamma.detach().clone().requires_grad_(), beta.detach().clone().requires_grad_()
    rm2, rv2 = torch.zeros(c, device=gpu), torch.ones(c, device=gpu)
    rr = bf(r).requires_grad_() if res else None
    yr = F.batch_norm(xr, rm2, rv2, g2, b2, True, 0.1, 1e-5)
    if res:
        yr = yr + rr
    if relu:
        yr = torch.relu(yr)
    assert rel_err(y.permute(0, 3, 1, 2), yr) < 1e-2
    assert rel_err(rm, rm2) < 1e-3 and rel_err(rv, rv2) < 1e-3
    gy = torch.randn_like(yr)
    yr.backward(gy)
    y.float().backward(gy.permute(0, 2, 3, 1))
    assert rel_err(xn.grad.permute(0, 3, 1, 2), xr.grad) < 2e-2
    assert rel_err(gamma.grad, g2.grad) < 2e-2
    assert rel_err(beta.grad, b2.grad) < 2e-2
    if res:
        assert rel_err(rn.grad.permute(0, 3, 1, 2), rr.grad) < 2e-2
    # the slice tickets are returned to 0 by each launch's last block: a second call is identical
    gamma.grad = None
    xn.grad = None
    y2 = OF.batch_norm(xn, gamma, beta, rm, rv, True, 0.1, 1e-5, rn, relu)
    assert torch.equal(y2, y)
    y2.float().backward(gy.permute(0, 2, 3, 1))
    assert rel_err(gamma.grad, g2.grad) < 2e-2
    assert OF._C().bn_error(True) == 0  # no one-launch BatchNorm wait timed out


@pytest.mark.parametrize("groups,n,c,h,res", [(4, 8, 64, 8, False), (4, 32, 256, 4, True), (2, 8, 512, 16, False),
                                                (8, 16, 2048, 4, True)])
def test_batchnorm_groups(gpu, groups, n, c, h, res):
    """Grouped BatchNorm (ops.functional.bn_groups): ONE launch per direction normalising `groups`
    micro-batches with their own statistics must equal `groups` separate BatchNorm calls: outputs and input
    gradients, running statistics after the `groups` in-order momentum updates, dgamma / dbeta
    as the sum over the groups."""
    torch.manual_seed(11)
    x = ((torch.randn(n, h, h, c, device=gpu) * 2 + torch.arange(n, device=gpu).view(n, 1, 1, 1) * 0.3)
         .bfloat16())
    r = torch.randn(n, h, h, c, device=gpu).bfloat16() if res else None
    gamma = torch.rand(c, device=gpu) + 0.5
    beta = torch.randn(c, device=gpu)
    gy = torch.randn(n, h, h, c, device=gpu).bfloat16()

    def run(grouped):
        rm, rv = torch.zeros(c, device=gpu), torch.ones(c, device=gpu)
        g_, b_ = gamma.clone().requires_grad_(), beta.clone().requires_grad_()
        xg = x.clone().requires_grad_()
        rg = r.clone().requires_grad_() if res else None
        if grouped:
            with OF.bn_groups(groups):
                y = OF.batch_norm(xg, g_, b_, rm, rv, True, 0.1, 1e-5, rg, True)
            y.backward(gy)
        else:
            ys = []
            for k, (xs, gs) in enumerate(zip(xg.chunk(groups), gy.chunk(groups))):
                ys.append(OF.batch_norm(xs, g_, b_, rm, rv, True, 0.1, 1e-5, rg.chunk(groups)[k] if res else None,
                                        True))
            y = torch.cat(ys)
            y.backward(gy)
        return y.detach(), xg.grad, (rg.grad if res else None), g_.grad, b_.grad, rm, rv

    a, b = run(True), run(False)
    # (the grouped launch cuts each group into fewer row chunks than a lone call: fp32 partial sums in a
    # different order, so bf16 outputs may differ by an ulp here and there)
    assert rel_err(a[0].float(), b[0].float()) < 2e-3, "forward"
    assert rel_err(a[1].float(), b[1].float()) < 2e-3, "dx"
    if res:
        assert rel_err(a[2].float(), b[2].float()) < 2e-3, "dres"
    for k, name in ((3, "dgamma"), (4, "dbeta"), (5, "running_mean"), (6, "running_var")):
        assert rel_err(a[k], b[k]) < 1e-4, name
    # and it is not the ungrouped BatchNorm: statistics over the whole batch give a different output
    with torch.no_grad():
        whole = OF.batch_norm(x, gamma, beta, torch.zeros(c, device=gpu), torch.ones(c, device=gpu), True, 0.1,
                              1e-5, r, True)
    assert rel_err(whole.float(), a[0].float()) > 1e-2
    assert OF._C().bn_error(True) == 0


def test_batchnorm_one_launch_graph_replays(gpu):
    """The one-launch BatchNorm kernels (stats -> ticket finalize -> generation flag -> apply) captured in
    a hipGraph: every replay counts the channel groups' flags up and must reproduce the eager results bit
    for bit (forward y, running stats trajectory, and backward dx / dgamma / dbeta / residual grad)."""
    torch.manual_seed(5)
    n, c, h = 8, 256, 8
    x = (torch.randn(n, h, h, c, device=gpu) * 2 + 0.5).bfloat16()
    r = torch.randn(n, h, h, c, device=gpu).bfloat16()
    gamma = torch.rand(c, device=gpu) + 0.5
    beta = torch.randn(c, device=gpu)
    gy = torch.randn(n, h, h, c, device=gpu).bfloat16()

    def step(rm, rv):
        xg, rg = x.clone().requires_grad_(), r.clone().requires_grad_()
        g_, b_ = gamma.clone().requires_grad_(), beta.clone().requires_grad_()
        y = OF.batch_norm(xg, g_, b_, rm, rv, True, 0.1, 1e-5, rg, True)
        y.backward(gy)
        return y.detach(), xg.grad, rg.grad, g_.grad, b_.grad

    rm0, rv0 = torch.zeros(c, device=gpu), torch.ones(c, device=gpu)
    eager = [step(rm0, rv0) for _ in range(3)]
    rm1, rv1 = torch.zeros(c, device=gpu), torch.ones(c, device=gpu)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step(torch.zeros(c, device=gpu), torch.ones(c, device=gpu))  # warm-up (allocates the ticket windows)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        outs = step(rm1, rv1)
    for k in range(3):
        g.replay()
        torch.cuda.synchronize()
        for a, b in zip(outs, eager[k]):
            assert torch.equal(a, b), k
    assert torch.equal(rm1, rm0) and torch.equal(rv1, rv0)
    assert OF._C().bn_error(True) == 0


# c = 16: 8-channel vector kernels; c = 10: scalar kernels (MNIST CNN channel counts)
@pytest.mark.parametrize("k,s,p,relu,c", [(3, 2, 1, False, 16), (2, 2, 0, True, 16), (3, 2, 1, True, 64),
                                          (2, 2, 0, True, 10), (3, 2, 1, False, 10)])
def test_maxpool(gpu, k, s, p, relu, c):
    torch.manual_seed(3)
    x = torch.randn(4, c, 12, 12, device=gpu)
    xn = bf(x).permute(0, 2, 3, 1).contiguous().bfloat16().requires_grad_()
    y = OF.max_pool2d(xn, k, s, p, relu)
    xr = bf(x).requires_grad_()
    yr = F.max_pool2d(xr, k, s, p)
    if relu:
        yr = torch.relu(yr)
    assert torch.allclose(y.permute(0, 3, 1, 2).float(), yr)
    g = torch.randn_like(yr)
    yr.backward(g)
    y.float().backward(g.permute(0, 2, 3, 1))
    assert rel_err(xn.grad.permute(0, 3, 1, 2), xr.grad) < 1e-2


def test_avgpool_and_losses(gpu):
    torch.manual_seed(4)
    x = torch.randn(8, 4, 4, 64, device=gpu).bfloat16().requires_grad_()
    y = OF.global_avg_pool_flat(x)
    assert rel_err(y, x.float().mean((1, 2))) < 1e-2
    y.float().sum().backward()
    assert torch.allclose(x.grad.float(), torch.full_like(x.float(), 1 / 16), atol=1e-3)

    logits = torch.randn(300, 10, device=gpu, requires_grad=True)
    tgt = torch.randint(0, 10, (300,), device=gpu)
    loss = OF.cross_entropy(logits, tgt)
    l2 = logits.detach().clone().requires_grad_()
    ref = F.cross_entropy(l2, tgt)
    assert abs(loss.item() - ref.item()) < 1e-4
    loss.backward()
    ref.backward()
    assert rel_err(logits.grad, l2.grad) < 1e-4

    lp = OF.log_softmax(logits.detach().clone().requires_grad_())
    assert rel_err(lp, F.log_softmax(logits.detach(), 1)) < 1e-5
    nl = OF.nll_loss(lp, tgt)
    assert abs(nl.item() - ref.item()) < 1e-4

    pred = torch.randn(32, 1000, device=gpu, requires_grad=True)
    t = torch.randn(32, 1000, device=gpu)
    m = OF.mse_loss(pred, t)
    p2 = pred.detach().clone().requires_grad_()
    mr = F.mse_loss(p2, t)
    assert abs(m.item() - mr.item()) < 1e-4
    m.backward()
    mr.backward()
    assert rel_err(pred.grad, p2.grad) < 1e-5


def test_dropout(gpu):
    x = torch.ones(64, 4, 4, 32, device=gpu).bfloat16().requires_grad_()
    y = OF.dropout(x, 0.5, True, channel=True)
    keep = (y.float() != 0)
    # channel mode: constant over spatial positions of one (n, c)
    assert torch.equal(keep, keep[:, :1, :1, :].expand_as(keep))
    frac = keep.float().mean().item()
    assert 0.4 < frac < 0.6
    assert torch.allclose(y.float()[keep], torch.full_like(y.float()[keep], 2.0))
    y.float().sum().backward()
    assert torch.equal(x.grad.float() != 0, keep)


@pytest.mark.parametrize("rows,D,L", [(100, 16, 40), (100, 16, 3000), (37, 7, 500), (64, 100, 700),
                                       (300000, 16, 400)])
def test_embedding_bag(gpu, rows, D, L):
    """Lane-grouped forward (D <= 32), wide rows, and both backward paths: the deterministic row-owner
    scan (bit-identical across runs) and the atomic path for large tables (rows * L > 2^26)."""
    torch.manual_seed(5)
    w = torch.randn(rows, D, device=gpu, requires_grad=True)
    idx = torch.randint(0, min(rows, 100), (L,), device=gpu)  # repeated rows: accumulation order matters
    off = torch.sort(torch.randint(0, L, (8,), device=gpu)).values
    off[0] = 0
    y = OF.embedding_bag_sum(w, idx, off)
    w2 = w.detach().clone().requires_grad_()
    yr = F.embedding_bag(idx, w2, off, mode="sum")
    assert rel_err(y, yr) < 1e-5
    g = torch.randn_like(yr)
    y.backward(g)
    yr.backward(g)
    assert rel_err(w.grad, w2.grad) < 1e-5
    if rows * L <= (1 << 26):
        g1 = w.grad.clone()
        w.grad = None
        OF.embedding_bag_sum(w, idx, off).backward(g)
        assert torch.equal(w.grad, g1)


@pytest.mark.parametrize("kind", ["sgd", "adam", "adamw"])
def test_fused_optimizers(gpu, kind):
    from pytorch_distributed_examples_amd.ops import optim as O

    torch.manual_seed(6)
    shapes = [(1024, 784), (1024,), (10, 1024), (10,), (7, 3, 5, 5)]
    ps = [torch.randn(*s, device=gpu) for s in shapes]
    ref = [p.detach().clone().requires_grad_() for p in ps]
    mine = [p.detach().clone().requires_grad_() for p in ps]
    if kind == "sgd":
        o1, o2 = O.FusedSGD(mine, lr=0.05, momentum=0.9), torch.optim.SGD(ref, lr=0.05, momentum=0.9)
    elif kind == "adam":
        o1, o2 = O.FusedAdam(mine, lr=1e-3), torch.optim.Adam(ref, lr=1e-3)
    else:
        o1, o2 = O.FusedAdamW(mine, lr=1e-2), torch.optim.AdamW(ref, lr=1e-2)
    for _ in range(3):
        gs = [torch.randn_like(p) for p in ps]
        for p, g in zip(mine, gs):
            p.grad = g.clone()
        for p, g in zip(ref, gs):
            p.grad = g.clone()
        o1.step()
        o2.step()
    for a, b in zip(mine, ref):
        assert rel_err(a, b) < 1e-5


@pytest.mark.parametrize("kind", ["sgd", "adam", "adamw"])
def test_fused_optimizers_views_and_device_step(gpu, kind):
    """Parameters that are unaligned views of one flat buffer (scalar path next to the vector path) and
    gradients updated in place, so the device-side step counter (not the host) drives bias correction."""
    from pytorch_distributed_examples_amd.ops import optim as O

    torch.manual_seed(7)
    sizes = [10, 5000, 7, 20, 3, 16000]
    flat = torch.randn(sum(sizes), device=gpu)
    mine = [t.view(-1) for t in flat.split(sizes)]
    for t in mine:
        t.requires_grad_()
    ref = [t.detach().clone().requires_grad_() for t in mine]
    gflat = torch.zeros_like(flat)
    for t, g in zip(mine, gflat.split(sizes)):
        t.grad = g
    if kind == "sgd":
        o1, o2 = O.FusedSGD(mine, lr=0.05, momentum=0.9), torch.optim.SGD(ref, lr=0.05, momentum=0.9)
    elif kind == "adam":
        o1, o2 = O.FusedAdam(mine, lr=1e-3), torch.optim.Adam(ref, lr=1e-3)
    else:
        o1, o2 = O.FusedAdamW(mine, lr=1e-2), torch.optim.AdamW(ref, lr=1e-2)
    for _ in range(4):
        gs = torch.randn_like(flat)
        gflat.copy_(gs)
        for p, g in zip(ref, gs.split(sizes)):
            p.grad = g.clone()
        o1.step()
        o2.step()
    for a, b in zip(mine, ref):
        assert rel_err(a, b) < 1e-5
    assert int(o1._dev[0]["step"][0].item()) == 4 and int(o1._dev[0]["step"][1].item()) == 0


def test_direct_grad_accumulation(gpu):
    """Weight-gradient kernels add into an existing .grad (conv OIHW epilogue, linear wgrad, bias colsum,
    BN finalize); post-accumulate-grad hooks still fire once per backward; results equal autograd's own
    accumulation."""
    from pytorch_distributed_examples_amd.ops import layers as L

    torch.manual_seed(3)
    conv = L.Conv2d(16, 24, 3, stride=2, padding=1).to(gpu)
    bn = L.BatchNorm2d(24).to(gpu)
    fc = L.Linear(24, 10).to(gpu)
    x = OF.to_native_image(torch.randn(4, 16, 12, 12, device=gpu))

    def loss():
        h = bn(conv(x), relu=True)
        return OF.mse_loss(fc(OF.global_avg_pool_flat(h), out_f32=True), torch.ones(4, 10, device=gpu))

    params = list(conv.parameters()) + list(bn.parameters()) + list(fc.parameters())
    with OF.direct_grad_accumulation(False):
        loss().backward()
        loss().backward()
    ref = [p.grad.clone() for p in params]
    for p in params:
        p.grad = torch.zeros_like(p)
    fired = []
    handles = [p.register_post_accumulate_grad_hook(lambda q: fired.append(q)) for p in params]
    loss().backward()
    loss().backward()
    for h in handles:
        h.remove()
    assert len(fired) == 2 * len(params)
    for p, r in zip(params, ref):
        assert rel_err(p.grad, r) < 1e-5


@pytest.mark.parametrize("cfg", [(4, 64, 16, 64, 1, 1, 0), (2, 24, 8, 40, 1, 1, 0)])
def test_pointwise_conv_dense_path(gpu, cfg):
    """1x1 / stride-1 convs take the dense-operand GEMM path (no gather): fwd, dgrad, wgrad."""
    test_conv_fwd_bwd(gpu, cfg)


@pytest.mark.parametrize("kind", ["sgd", "adam"])
def test_optimizer_maintained_compute_copies(gpu, kind):
    """The fused optimizer writes the bf16 compute copies of linear and 1x1-conv weights in the same launch
    as the update, and both GEMM layouts of KxK conv weights in one batched launch after it; they equal a
    fresh conversion of the updated fp32 weights, an outside write (load_state_dict)
    is picked up through the version counter, and a 1x1 conv's dgrad reading the forward copy transposed
    matches the dgrad-layout path."""
    from pytorch_distributed_examples_amd.ops import layers as L
    from pytorch_distributed_examples_amd.ops.optim import FusedAdam, FusedSGD

    torch.manual_seed(4)
    conv = L.Conv2d(32, 48, 1, bias=False).to(gpu)
    conv3 = L.Conv2d(3, 20, 3, padding=1).to(gpu)  # KxK: layout copies refreshed after the update
    conv3b = L.Conv2d(40, 72, 3, padding=1, bias=False).to(gpu)  # several 32 x 32 tiles, partial edge tiles
    fc = L.Linear(40, 12).to(gpu)
    params = list(conv.parameters()) + list(conv3.parameters()) + list(conv3b.parameters()) + list(fc.parameters())
    opt = (FusedSGD(params, lr=0.1, momentum=0.9) if kind == "sgd" else FusedAdam(params, lr=1e-2))
    for p in params:
        p.grad = torch.randn_like(p)
    for _ in range(3):
        opt.step()
    assert torch.equal(OF._maintained(conv.weight, "conv_fwd"), conv.weight.detach().view(48, 32).bfloat16())
    assert torch.equal(OF._maintained(fc.weight, "bf16"), fc.weight.detach().bfloat16())
    # KxK conv (3 -> 20 channels, padded to 8 / 24): both GEMM layouts refreshed by the one batched launch
    C = OF._C()
    w3 = conv3.weight.detach()
    assert torch.equal(OF._maintained(conv3.weight, "conv_fwd"), C.conv_w_fwd(w3, 8, 24))
    assert torch.equal(OF._maintained(conv3.weight, "conv_dgrad"), C.conv_w_dgrad(w3, 8, 24))
    w3b = conv3b.weight.detach()
    assert torch.equal(OF._maintained(conv3b.weight, "conv_fwd"), C.conv_w_fwd(w3b, 40, 72))
    assert torch.equal(OF._maintained(conv3b.weight, "conv_dgrad"), C.conv_w_dgrad(w3b, 40, 72))
    sd3 = {k: torch.randn_like(v) for k, v in conv3.state_dict().items()}
    conv3.load_state_dict(sd3)
    assert torch.equal(OF._maintained(conv3.weight, "conv_dgrad"), C.conv_w_dgrad(sd3["weight"], 8, 24))
    sd = {k: torch.randn_like(v) for k, v in conv.state_dict().items()}
    conv.load_state_dict(sd)
    assert torch.equal(OF._maintained(conv.weight, "conv_fwd"), sd["weight"].view(48, 32).bfloat16())
    dy = torch.randn(2, 5, 5, 48, device=gpu).bfloat16()
    wf = OF._maintained(conv.weight, "conv_fwd")
    a = C.conv_dgrad(dy, wf, 5, 5, 1, 1, 1, 0, None, True)
    b = C.conv_dgrad(dy, C.conv_w_dgrad(conv.weight.detach(), 32, 48), 5, 5, 1, 1, 1, 0)
    assert rel_err(a, b) < 1e-3
    # strided 1x1 (ResNet downsample): same transposed read, dy gathered at stride 2 (dx 10x10)
    a2 = C.conv_dgrad(dy, wf, 10, 10, 1, 1, 2, 0, None, True)
    b2 = C.conv_dgrad(dy, C.conv_w_dgrad(conv.weight.detach(), 32, 48), 10, 10, 1, 1, 2, 0)
    assert rel_err(a2, b2) < 1e-3


def test_inkernel_splitk_path(gpu):
    """The opt-in in-launch split-K combine (gemm.hip write_slab_and_reduce, PDE_GEMM_INKERNEL_SPLITK=1)
    is read once per process, so the linear and conv shape tests rerun in a child with it on."""
    import os
    import subprocess
    import sys

    here = os.path.abspath(__file__)
    env = dict(os.environ, PDE_GEMM_INKERNEL_SPLITK="1")
    res = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", "--timeout", "120",
                          f"{here}::test_linear_fwd_bwd", f"{here}::test_conv_fwd_bwd"],
                         env=env, capture_output=True, text=True, timeout=300, cwd=os.path.dirname(os.path.dirname(here)))
    assert res.returncode == 0, res.stdout[-3000:] + res.stderr[-3000:]


def test_first_write_after_zero_grad_stores(gpu):
    """DDP.zero_grad marks the flat gradient's views freshly zeroed; the first weight-gradient kernel of the step
    then stores instead of adding (no read-modify-write), later kernels of the same step add.  Garbage planted in
    the buffer AFTER zero_grad is overwritten by the first backward; a second backward accumulates."""
    from pytorch_distributed_examples_amd.ops import layers as L
    from pytorch_distributed_examples_amd.parallel.ddp import DistributedDataParallel

    torch.manual_seed(5)
    conv = L.Conv2d(16, 24, 3, stride=1, padding=1).to(gpu)
    conv1 = L.Conv2d(24, 32, 1).to(gpu)
    bn = L.BatchNorm2d(32).to(gpu)
    fc = L.Linear(32, 10).to(gpu)
    model = torch.nn.ModuleList([conv, conv1, bn, fc])
    x = OF.to_native_image(torch.randn(4, 16, 12, 12, device=gpu))

    def loss():
        h = bn(conv1(conv(x)), relu=True)
        return OF.mse_loss(fc(OF.global_avg_pool_flat(h), out_f32=True), torch.ones(4, 10, device=gpu))

    params = list(model.parameters())
    with OF.direct_grad_accumulation(False):
        for p in params:
            p.grad = None
        loss().backward()
    ref1 = [p.grad.clone() for p in params]
    ddp = DistributedDataParallel(model, overlap=False)
    ddp.zero_grad()
    weights = [conv.weight, conv1.weight, fc.weight]
    for w in weights:
        w.grad.fill_(123.0)  # would survive a read-modify-write; a first write must replace it
    loss().backward()
    for p, r in zip(params, ref1):
        if any(p is w for w in weights):
            assert rel_err(p.grad, r) < 1e-5
    for w in weights:
        assert "_pde_fresh" not in w.grad.__dict__
    loss().backward()  # same step, no zero_grad: adds
    for p, r in zip(params, ref1):
        if any(p is w for w in weights):
            assert rel_err(p.grad, 2 * r) < 1e-5


def test_static_graph_ddp_skips_the_zero_fill(gpu):
    """DDP(static_graph=True): every gradient of a conv / BatchNorm / linear model is first written by a storing
    kernel (conv and linear weight + bias gradients, BatchNorm's dgamma / dbeta finalize), so from the third step
    on zero_grad skips the flat-gradient fill -- and the trained weights are bitwise those of the filling DDP."""
    from pytorch_distributed_examples_amd.ops import layers as L
    from pytorch_distributed_examples_amd.ops.optim import FusedSGD
    from pytorch_distributed_examples_amd.parallel.ddp import DistributedDataParallel

    def make():
        torch.manual_seed(6)
        return torch.nn.ModuleList([L.Conv2d(16, 24, 3, stride=1, padding=1), L.BatchNorm2d(24),
                                    L.Conv2d(24, 32, 1, bias=False), L.BatchNorm2d(32), L.Linear(32, 10)]).to(gpu)

    runs = []
    for static in (False, True):
        m = make()
        ddp = DistributedDataParallel(m, overlap=False, static_graph=static)
        opt = FusedSGD(m.parameters(), lr=0.05, momentum=0.9)
        for step in range(5):
            g = torch.Generator(device="cpu").manual_seed(step)
            x = OF.to_native_image(torch.randn(4, 16, 12, 12, generator=g).to(gpu))
            ddp.zero_grad()
            if static and step >= 2:
                ddp.flat_grad.fill_(77.0)  # what a skipped fill leaves behind must not matter
            h = m[1](m[0](x), relu=True)
            h = m[3](m[2](h), relu=True)
            loss = OF.mse_loss(m[4](OF.global_avg_pool_flat(h), out_f32=True), torch.ones(4, 10, device=gpu))
            loss.backward()
            opt.step()
        torch.cuda.synchronize()
        runs.append((m, ddp))
    (ma, _), (mb, db) = runs
    assert db.fills_skipped == 3, db.fills_skipped
    for pa, pb in zip(ma.parameters(), mb.parameters()):
        assert torch.equal(pa, pb) and torch.equal(pa.grad, pb.grad)


@pytest.mark.parametrize("M,K,N,bias,relu", [(32768, 64, 256, False, False), (8192, 128, 512, False, False),
                                             (5000, 64, 64, True, True), (4100, 40, 200, True, False),
                                             (6000, 56, 384, False, True), (4096, 32, 128, True, True)])
def test_lowk_gemm_path(gpu, M, K, N, bias, relu):
    """K <= 64 with dense K-contiguous operands and >= 4096 rows: the streamed low-K kernel (gemm_lowk.h: the B
    strip through LDS into per-wave registers, A fragments straight from global memory, transposed MFMAs, output
    staged per wave and stored as 16-byte rows) -- 128- and 64-wide strips, K not a multiple of 32, ragged M / N
    edges, bias / ReLU epilogues; bitwise deterministic across launches.  (8192x512x128: the tile core, K > 64.)"""
    C = OF._C()
    torch.manual_seed(7)
    x = torch.randn(M, K, device=gpu).bfloat16()
    w = (torch.randn(N, K, device=gpu) * 0.1).bfloat16()
    b = torch.randn(N, device=gpu) if bias else None
    y = C.linear_fwd(x, w, b, relu, False)
    ref = x.float() @ w.float().t()
    if bias:
        ref = ref + b
    if relu:
        ref = torch.relu(ref)
    assert y.shape == (M, N) and y.dtype == torch.bfloat16
    assert rel_err(y, ref) < 1e-2
    assert (y.float() - ref).abs().max().item() < 0.05 * ref.abs().max().item() + 1e-2
    assert torch.equal(y, C.linear_fwd(x, w, b, relu, False))


def test_lowk_gemm_path_k128_subprocess(gpu):
    """The low-K kernel's KT = 3 / 4 instantiations (K up to 128), enabled with PDE_GEMM_LOWK_MAX_K=128 in a child
    process (the dispatch policy is read once per process)."""
    import os
    import subprocess
    import sys

    code = (
        "import torch\n"
        "from pytorch_distributed_examples_amd.ops import functional as OF\n"
        "C = OF._C(); torch.manual_seed(3)\n"
        "for M, K, N in ((6000, 96, 384), (8192, 128, 512), (4096, 128, 200)):\n"
        "    x = torch.randn(M, K, device='cuda').bfloat16(); w = (torch.randn(N, K, device='cuda') * 0.1).bfloat16()\n"
        "    b = torch.randn(N, device='cuda')\n"
        "    y = C.linear_fwd(x, w, b, True, False)\n"
        "    ref = torch.relu(x.float() @ w.float().t() + b)\n"
        "    e = ((y.float() - ref).norm() / ref.norm()).item()\n"
        "    assert e < 1e-2, (M, K, N, e)\n"
        "    assert torch.equal(y, C.linear_fwd(x, w, b, True, False))\n"
        "print('LOWK128_OK')\n")
    env = dict(os.environ, PDE_GEMM_LOWK_MAX_K="128", PDE_GEMM_LOG="1")
    res = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120,
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert res.returncode == 0 and "LOWK128_OK" in res.stdout, res.stderr[-3000:]
    assert res.stderr.count("[gemm] lowk") >= 3, res.stderr[-2000:]


@pytest.mark.parametrize("n,h,ci,co,k", [(8, 4, 512, 512, 3), (8, 8, 256, 256, 3), (8, 4, 2048, 512, 1),
                                          (2, 4, 512, 2048, 1)])
def test_deferred_conv_slabs_into_batchnorm(gpu, n, h, ci, co, k):
    """A split-K conv whose slabs the one-launch BatchNorm sums itself (bn_follows: the stage-2 layers at m = 8,
    where the batched slab loads of k_bn_fwd_fused run) gives the same activation and running statistics as the
    conv reducing its own slabs first, and matches an fp32 conv + BatchNorm."""
    torch.manual_seed(11)
    x = OF.to_native_image(torch.randn(n, ci, h, h, device=gpu))
    w = torch.randn(co, ci, k, k, device=gpu) * (1.0 / (ci * k * k) ** 0.5)
    g = torch.rand(co, device=gpu) + 0.5
    b = torch.randn(co, device=gpu) * 0.1
    outs = []
    for defer in (True, False):
        rm, rv = torch.zeros(co, device=gpu), torch.ones(co, device=gpu)
        y = OF.conv2d(x, w, None, 1, k // 2, bn_follows=defer)
        z = OF.batch_norm(y, g, b, rm, rv, True, relu=True)
        torch.cuda.synchronize()
        outs.append((z.clone(), rm.clone(), rv.clone()))
    OF.check_device_errors("deferred slabs")
    # (the standalone slab reduction sums with several slab lanes per column for > 2 slabs, the BatchNorm in slab
    # order: the bf16 activations may differ in the last bit, the statistics by fp32 rounding)
    assert (outs[0][0].float() - outs[1][0].float()).abs().max().item() <= 2e-2 * outs[1][0].float().abs().max().item()
    torch.testing.assert_close(outs[0][1], outs[1][1], rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(outs[0][2], outs[1][2], rtol=1e-3, atol=1e-4)
    ref = torch.relu(torch.nn.functional.batch_norm(
        torch.nn.functional.conv2d(x[..., :ci].permute(0, 3, 1, 2).float(), w.bfloat16().float(), padding=k // 2),
        None, None, g, b, True, 0.1, 1e-5))
    got = outs[0][0][..., :co].permute(0, 3, 1, 2).float()
    assert rel_err(got, ref) < 2e-2
