"""Model-level GPU checks: one forward/backward of each model family on the native path against the
CPU fp32 reference path of the SAME module (same weights), and loss decrease over a few steps."""
import copy

import pytest
import torch

from pytorch_distributed_examples_amd.models.cnn import Net
from pytorch_distributed_examples_amd.models.mlp import MLP
from pytorch_distributed_examples_amd.models.resnet import ResNetShard1, ResNetShard2
from pytorch_distributed_examples_amd.ops import functional as OF

pytestmark = pytest.mark.gpu


def rel_err(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def test_mlp_step_matches_cpu(gpu):
    torch.manual_seed(0)
    m_cpu = MLP(hidden_layers=5, features=1024)
    m_gpu = copy.deepcopy(m_cpu).to(gpu)
    x = torch.randn(128, 1, 28, 28)
    y = torch.randint(0, 10, (128,))
    with OF.emulate_bf16_on_cpu():
        l_cpu = OF.cross_entropy(m_cpu(x), y)
        l_cpu.backward()
    l_gpu = OF.cross_entropy(m_gpu(x.to(gpu)), y.to(gpu))
    l_gpu.backward()
    assert abs(l_cpu.item() - l_gpu.item()) < 2e-2
    for (n, p1), p2 in zip(m_cpu.named_parameters(), m_gpu.parameters()):
        assert rel_err(p2.grad.cpu(), p1.grad) < 5e-2, n


@pytest.mark.parametrize("batch", [128, 37])
def test_fused_mlp_matches_cpu(gpu, batch):
    """models/mlp_fused.py (explicit launch sequence, bias gradient through the ones column) against the
    CPU fp32 reference of the same weights; odd batch = unaligned ld and partial tiles."""
    from pytorch_distributed_examples_amd.models.mlp_fused import FusedMLP

    torch.manual_seed(0)
    m_cpu = MLP(hidden_layers=5, features=1024)
    m_gpu = copy.deepcopy(m_cpu).to(gpu)
    x = torch.randn(batch, 1, 28, 28)
    y = torch.randint(0, 10, (batch,))
    with OF.emulate_bf16_on_cpu():
        l_cpu = OF.cross_entropy(m_cpu(x), y)
        l_cpu.backward()
    f = FusedMLP(m_gpu)
    l_gpu = f.forward_backward(x.to(gpu), y.to(gpu))
    assert abs(l_cpu.item() - l_gpu.item()) < 2e-2
    for (n, p1), p2 in zip(m_cpu.named_parameters(), m_gpu.parameters()):
        assert rel_err(p2.grad.cpu(), p1.grad) < 5e-2, n
    # accumulate adds, a second plain call overwrites
    g1 = [p.grad.clone() for p in m_gpu.parameters()]
    f.forward_backward(x.to(gpu), y.to(gpu), accumulate=True)
    for p, g in zip(m_gpu.parameters(), g1):
        assert torch.allclose(p.grad, 2 * g, rtol=1e-4, atol=1e-6)
    f.forward_backward(x.to(gpu), y.to(gpu))
    for p, g in zip(m_gpu.parameters(), g1):
        assert torch.allclose(p.grad, g, rtol=1e-5, atol=1e-7)


def test_fused_mlp_trains_with_adam(gpu):
    from pytorch_distributed_examples_amd.models.mlp_fused import FusedMLP
    from pytorch_distributed_examples_amd.ops.optim import FusedAdam

    torch.manual_seed(0)
    m = MLP(hidden_layers=5, features=1024).to(gpu)
    f = FusedMLP(m)
    opt = FusedAdam(m.parameters(), lr=1e-3)
    x = torch.randn(128, 1, 28, 28, device=gpu)
    y = torch.randint(0, 10, (128,), device=gpu)
    losses = []
    for _ in range(20):
        losses.append(f.forward_backward(x, y).item())
        opt.step()
    assert losses[-1] < 0.5 * losses[0], losses
    # the layer-by-layer path sees the trained weights (bf16 copies maintained by the optimizer)
    assert abs(OF.cross_entropy(m(x), y).item() - f.forward_backward(x, y).item()) < 1e-3


def test_cnn_step_matches_cpu(gpu):
    torch.manual_seed(0)
    m_cpu = Net().eval()  # eval: dropout off so both paths are deterministic
    m_gpu = copy.deepcopy(m_cpu).to(gpu).eval()
    x = torch.randn(64, 1, 28, 28)
    y = torch.randint(0, 10, (64,))
    with OF.emulate_bf16_on_cpu():
        l_cpu = OF.nll_loss(m_cpu(x), y)
        l_cpu.backward()
    l_gpu = OF.nll_loss(m_gpu(x.to(gpu)), y.to(gpu))
    l_gpu.backward()
    assert abs(l_cpu.item() - l_gpu.item()) < 2e-2
    for (n, p1), p2 in zip(m_cpu.named_parameters(), m_gpu.parameters()):
        assert rel_err(p2.grad.cpu(), p1.grad) < 5e-2, n


def test_resnet_shards_match_cpu(gpu):
    torch.manual_seed(0)
    s1, s2 = ResNetShard1(), ResNetShard2()
    g1, g2 = copy.deepcopy(s1).to(gpu), copy.deepcopy(s2).to(gpu)
    x = torch.randn(4, 3, 128, 128)
    t = torch.randn(4, 1000)
    with OF.emulate_bf16_on_cpu():
        out_cpu = s2(s1(x))
    out_gpu = g2(g1(x.to(gpu)))
    assert out_gpu.shape == (4, 1000)
    # 53 bf16-stored layers with batch-4 BatchNorm: rounding noise compounds end to end (the per-block
    # test below holds each block to 3%)
    assert rel_err(out_gpu.cpu(), out_cpu) < 0.12
    with OF.emulate_bf16_on_cpu():
        OF.mse_loss(out_cpu, t).backward()
    OF.mse_loss(out_gpu, t.to(gpu)).backward()
    # gradients near the loss only: deeper ones go through up to 50 batch-4 BatchNorm backwards, where bf16
    # noise is amplified chaotically (test_resnet_blocks_backward_match_cpu checks every block on its own).
    # The last BN's gamma gradient (sum dy * xhat over 4 x 4 x 4 positions per channel) inherits the ~10 %
    # end-to-end forward noise of xhat, measured 0.18 on MI355X.
    for (n, p1), p2 in zip(list(s2.named_parameters())[-4:], list(g2.parameters())[-4:]):
        assert rel_err(p2.grad.cpu(), p1.grad) < (0.3 if "bn" in n else 0.15), n


def test_resnet_blocks_grouped_bn_match_microbatches(gpu):
    """A pipeline unit of 4 micro-batches with grouped BatchNorm (one launch sequence, per-micro-batch
    statistics; conv -> BN split-K slab path included) against the same block run micro-batch by
    micro-batch: outputs, input gradients and parameter gradients agree to bf16 noise."""
    torch.manual_seed(3)
    s1, s2 = ResNetShard1(), ResNetShard2()
    blocks = [s1.seq[4][0], s1.seq[5][0], s2.seq[0][0], s2.seq[1][1]]
    shapes = [(64, 32), (256, 32), (512, 16), (2048, 4)]
    G, m = 4, 4
    for blk, (c, hw) in zip(blocks, shapes):
        x = torch.randn(G * m, hw, hw, c).to(torch.bfloat16).to(gpu)
        gy = None
        outs = []
        for grouped in (True, False):
            b = copy.deepcopy(blk).to(gpu)
            xg = x.clone().requires_grad_()
            if grouped:
                with OF.bn_groups(G):
                    y = b(xg)
                gen = torch.Generator().manual_seed(c)
                gy = torch.randn(y.shape, generator=gen).to(torch.bfloat16).to(gpu)
                y.backward(gy)
            else:
                ys = [b(xs) for xs in xg.split(m)]
                torch.cat(ys).backward(gy)
                y = torch.cat(ys)
            grads = torch.cat([p.grad.float().reshape(-1) for p in b.parameters()])
            bufs = torch.cat([t.float().reshape(-1) for n, t in b.named_buffers() if "running" in n])
            outs.append((y.detach().float(), xg.grad.float(), grads, bufs))
        (ya, da, ga, ba), (yb, db, gb, bb) = outs
        assert rel_err(ya, yb) < 1e-2, (c, rel_err(ya, yb))
        assert rel_err(da, db) < 3e-2, (c, rel_err(da, db))
        assert rel_err(ga, gb) < 3e-2, (c, rel_err(ga, gb))
        assert rel_err(ba, bb) < 1e-3, (c, rel_err(ba, bb))


def test_resnet_blocks_match_cpu(gpu):
    """Each bottleneck (with and without downsample / stride) on the same bf16 input: GPU NHWC vs CPU NCHW."""
    torch.manual_seed(0)
    s1, s2 = ResNetShard1(), ResNetShard2()
    blocks = [s1.seq[4][0], s1.seq[4][1], s1.seq[5][0], s2.seq[0][0], s2.seq[1][0], s2.seq[1][2]]
    shapes = [(64, 32), (256, 32), (256, 32), (512, 16), (1024, 8), (2048, 4)]
    for blk, (c, hw) in zip(blocks, shapes):
        x = torch.randn(4, c, hw, hw).to(torch.bfloat16).float()
        g = copy.deepcopy(blk).to(gpu)
        with OF.emulate_bf16_on_cpu():
            ref = blk(x)
        out = g(x.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).to(gpu))
        out = out.float().permute(0, 3, 1, 2).cpu()
        assert out.shape == ref.shape
        assert rel_err(out, ref) < 3e-2, (c, hw, rel_err(out, ref))


def test_resnet_blocks_backward_match_cpu(gpu):
    """Backward of each bottleneck from the same upstream gradient: input grad and every conv / BN
    parameter grad, GPU NHWC kernels vs the bf16-emulating CPU reference."""
    torch.manual_seed(0)
    s1, s2 = ResNetShard1(), ResNetShard2()
    blocks = [s1.seq[4][0], s1.seq[5][0], s1.seq[5][1], s2.seq[0][0], s2.seq[1][0], s2.seq[1][2]]
    shapes = [(64, 32), (256, 32), (512, 16), (512, 16), (1024, 8), (2048, 4)]
    for blk, (c, hw) in zip(blocks, shapes):
        x = torch.randn(8, c, hw, hw).to(torch.bfloat16).float().requires_grad_()
        g = copy.deepcopy(blk).to(gpu)
        with OF.emulate_bf16_on_cpu():
            ref = blk(x)
        up = torch.randn_like(ref).to(torch.bfloat16).float()
        ref.backward(up)
        xg = x.detach().permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).to(gpu).requires_grad_()
        out = g(xg)
        (out.float() * up.permute(0, 2, 3, 1).to(gpu)).sum().backward()
        errs = {"x": rel_err(xg.grad.float().permute(0, 3, 1, 2).cpu(), x.grad)}
        for (n, p1), p2 in zip(blk.named_parameters(), g.parameters()):
            errs[n] = rel_err(p2.grad.cpu(), p1.grad)
        bad = {k: v for k, v in errs.items() if v > 5e-2}
        assert not bad, (c, hw, errs)


def test_cnn_trains(gpu):
    from pytorch_distributed_examples_amd.data.synthetic import SyntheticMNIST
    from pytorch_distributed_examples_amd.ops.optim import FusedSGD

    torch.manual_seed(0)
    m = Net().to(gpu)
    opt = FusedSGD(m.parameters(), lr=0.05, momentum=0.9)
    data = SyntheticMNIST(4096, device=gpu, seed=1)
    losses = []
    for i in range(30):
        x, y = data.batch(i, 256)
        opt.zero_grad(set_to_none=False)
        loss = OF.nll_loss(m(x), y)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert sum(losses[-5:]) / 5 < losses[0] * 0.7, losses


def _mixed_reference_loss(m, x, y, mask2=None, mask1=None):
    """``mask2`` [N, 20] (Dropout2d, already x 1/(1-p)) on conv2's output, ``mask1`` [N, 50] on relu(fc1)."""
    import torch.nn.functional as F

    def st(t):  # bf16-rounded value, identity gradient
        return t + (t.detach().to(torch.bfloat16).float() - t.detach())

    c1 = F.conv2d(st(x), st(m.conv1.weight), m.conv1.bias)
    r1 = st(F.relu(F.max_pool2d(c1, 2)))
    c2 = F.conv2d(r1, st(m.conv2.weight), m.conv2.bias)
    if mask2 is not None:
        c2 = c2 * mask2[:, :, None, None]
    r2 = F.relu(F.max_pool2d(c2, 2)).flatten(1)
    h = F.relu(F.linear(r2, m.fc1.weight, m.fc1.bias))
    if mask1 is not None:
        h = h * mask1
    return F.nll_loss(F.log_softmax(F.linear(h, m.fc2.weight, m.fc2.bias), 1), y)


def _cnn_hash_u01(seed: int, ids):
    """Host copy of cnn_fused.hip's counter hash (splitmix64 finaliser over seed + golden * (id + 1))."""
    import numpy as np

    with np.errstate(over="ignore"):
        z = np.uint64(seed) + np.uint64(0x9E3779B97F4A7C15) * (np.asarray(ids, dtype=np.uint64) + np.uint64(1))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z >> np.uint64(40)).astype(np.float64) / 16777216.0


def _cnn_masks(counter: int, n: int, p2: float, p1: float):
    """The training kernel's Dropout2d [n, 20] and dropout [n, 50] multipliers for RNG counter ``counter``."""
    import numpy as np

    seed = (counter * 0xD1B54A32D192ED03) % (1 << 64)
    u2 = _cnn_hash_u01(seed ^ 0x5BD1E995, np.arange(n * 20)).reshape(n, 20)
    u1 = _cnn_hash_u01(seed ^ 0x27D4EB2F, np.arange(n * 50)).reshape(n, 50)
    m2 = np.where(u2 >= np.float32(p2), np.float32(1.0) / np.float32(1.0 - p2), 0.0).astype(np.float32)
    m1 = np.where(u1 >= np.float32(p1), np.float32(1.0) / np.float32(1.0 - p1), 0.0).astype(np.float32)
    return torch.from_numpy(m2), torch.from_numpy(m1)


@pytest.mark.parametrize("p2,p1", [(0.5, 0.5), (0.25, 0.6)])
def test_fused_cnn_dropout_masks(gpu, p2, p1):
    """Training-mode dropout of the headline kernel (cnn_fused.hip P0/P2/P3): the kernel's loss and every
    gradient must match a CPU reference that applies the SAME hash masks -- Dropout2d constant per (image,
    channel) on conv2's output, elementwise dropout on relu(fc1), both scaled by 1/(1-p) and the same in
    forward and backward.  Also: keep rates within 2 % of 1-p, a wrong seed does NOT match (the check
    discriminates), and successive hipGraph replays draw fresh masks (the counter advances per step)."""
    from pytorch_distributed_examples_amd.models.cnn_fused import FusedCNN

    torch.manual_seed(0)
    n = 512
    m_cpu = Net().train()
    m_gpu = copy.deepcopy(m_cpu).to(gpu).train()
    fused = FusedCNN(m_gpu)
    x = torch.randn(n, 1, 28, 28)
    y = torch.randint(0, 10, (n,))
    xg, yg = x.to(gpu), y.to(gpu)
    ctr = OF._rng_counter(xg.device)
    ctr.fill_(12345)

    m2, m1 = _cnn_masks(12345, n, p2, p1)
    assert abs((m2 > 0).float().mean().item() - (1 - p2)) < 0.02
    assert abs((m1 > 0).float().mean().item() - (1 - p1)) < 0.02

    def reference(mask2, mask1):
        ref = copy.deepcopy(m_cpu)
        loss = _mixed_reference_loss(ref, x, y, mask2, mask1)
        loss.backward()
        return loss.item(), torch.cat([p.grad.reshape(-1) for p in ref.parameters()])

    def errs(g, ref_g):
        out, off = {}, 0
        for name, p in m_cpu.named_parameters():
            k = p.numel()
            out[name] = rel_err(g[off:off + k].cpu(), ref_g[off:off + k])
            off += k
        return out

    g = torch.zeros(fused.flat.numel(), device=gpu)
    loss = fused.forward_backward(xg, yg, grad_out=g, p_drop2=p2, p_drop1=p1).item()
    assert int(ctr.item()) == 12346  # the reduction advanced the counter for the next step
    l_ref, g_ref = reference(m2, m1)
    assert abs(loss - l_ref) < 1e-2, (loss, l_ref)
    e = errs(g, g_ref)
    assert all(v < 3e-2 for v in e.values()), e
    # negative control: the next counter's masks must NOT explain this step
    w2, w1 = _cnn_masks(12346, n, p2, p1)
    l_w, g_w = reference(w2, w1)
    assert max(errs(g, g_w).values()) > 0.2

    # hipGraph: one captured step, two replays -> masks of counters 12346 and 12347
    ctr.fill_(12346)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fused.forward_backward(xg, yg, grad_out=g, p_drop2=p2, p_drop1=p1)  # warm-up: counter -> 12347
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        gl = fused.forward_backward(xg, yg, grad_out=g, p_drop2=p2, p_drop1=p1)
    ctr.fill_(12346)
    for k in (12346, 12347):
        graph.replay()
        torch.cuda.synchronize()
        l_ref, g_ref = reference(*_cnn_masks(k, n, p2, p1))
        assert abs(gl.item() - l_ref) < 1e-2, (k, gl.item(), l_ref)
        e = errs(g, g_ref)
        assert all(v < 3e-2 for v in e.values()), (k, e)
    assert int(ctr.item()) == 12348


def test_fused_cnn_matches_reference(gpu):
    """Fused whole-network kernel (bf16 MFMA convs, fp32 accumulate / head) vs a CPU fp32 reference that
    rounds the same operands to bf16 (straight-through, so gradients stay fp32), dropout off (eval).
    With identical conv inputs the max-pool argmax decisions agree; against the plain fp32 model ~1% of
    pooling windows pick another tap, which moves whole gradient contributions (~10% relative error on
    the conv1 weight gradient, as measured)."""
    from pytorch_distributed_examples_amd.models.cnn_fused import FusedCNN

    torch.manual_seed(0)
    m_cpu = Net().eval()
    m_gpu = copy.deepcopy(m_cpu).to(gpu).eval()
    fused = FusedCNN(m_gpu)
    x = torch.randn(300, 1, 28, 28)
    y = torch.randint(0, 10, (300,))
    l_cpu = _mixed_reference_loss(m_cpu, x, y)
    l_cpu.backward()
    g = torch.zeros(fused.flat.numel(), device=gpu)
    loss = fused.forward_backward(x.to(gpu), y.to(gpu), grad_out=g)
    assert abs(loss.item() - l_cpu.item()) < 1e-2
    off, errs = 0, {}
    for n, p in m_cpu.named_parameters():
        k = p.numel()
        errs[n] = rel_err(g[off:off + k].cpu().view_as(p), p.grad)
        off += k
    assert all(v < 3e-2 for v in errs.values()), errs


@pytest.mark.parametrize("mode", ["reduce", "sgd_step"])
def test_fused_cnn_sgd_matches_optimizer(gpu, mode):
    """The fused SGD update (in the slab reduction, or the post-all-reduce cnn_sgd kernel) refreshes the
    bf16 fragment image in place of the prep kernel: weights and losses must track the generic path
    (prep every step + FusedSGD) bit for bit over several steps (eval mode: no dropout)."""
    from pytorch_distributed_examples_amd.models.cnn_fused import FusedCNN
    from pytorch_distributed_examples_amd.ops.optim import FusedSGD

    torch.manual_seed(0)
    m_ref = Net().to(gpu).eval()
    m_fus = copy.deepcopy(m_ref)
    f_ref, f_fus = FusedCNN(m_ref), FusedCNN(m_fus)
    g_ref, g_fus = f_ref.grad_buffer(), f_fus.grad_buffer()
    o_ref, o_fus = FusedSGD(m_ref.parameters(), lr=0.05), FusedSGD(m_fus.parameters(), lr=0.05)
    x = torch.randn(6, 256, 1, 28, 28, device=gpu)
    y = torch.randint(0, 10, (6, 256), device=gpu)
    # the reference runs first: its optimiser steps bump the (global) weight generation, which would
    # otherwise make the fused model re-prep and hide the fragment-refresh path under test
    l_ref = []
    for i in range(6):
        l_ref.append(f_ref.forward_backward(x[i], y[i], grad_out=g_ref).item())
        o_ref.step()
    for i in range(6):
        if mode == "reduce":
            l_fus = f_fus.forward_backward(x[i], y[i], grad_out=g_fus, sgd=o_fus)
        else:
            l_fus = f_fus.forward_backward(x[i], y[i], grad_out=g_fus)
            f_fus.sgd_step(o_fus, g_fus)
        assert i == 0 or f_fus._frag_gen is not None
        assert l_ref[i] == l_fus.item(), (i, l_ref[i], l_fus.item())
    torch.cuda.synchronize()
    assert torch.equal(f_ref.flat, f_fus.flat)
    # an external write must be picked up after invalidate()
    with torch.no_grad():
        m_fus.conv1.weight.mul_(0.5)
        m_ref.conv1.weight.mul_(0.5)
    f_fus.invalidate()
    f_ref.invalidate()
    l_ref = f_ref.forward_backward(x[0], y[0], grad_out=g_ref)
    l_fus = f_fus.forward_backward(x[0], y[0], grad_out=g_fus)
    assert l_ref.item() == l_fus.item()


def test_fused_cnn_trains_with_dropout(gpu):
    from pytorch_distributed_examples_amd.data.synthetic import SyntheticMNIST
    from pytorch_distributed_examples_amd.models.cnn_fused import FusedCNN
    from pytorch_distributed_examples_amd.ops.optim import FusedSGD

    torch.manual_seed(0)
    m = Net().to(gpu).train()
    fused = FusedCNN(m)
    fused.grad_buffer()
    opt = FusedSGD(m.parameters(), lr=0.05, momentum=0.9)
    data = SyntheticMNIST(4096, device=gpu, seed=1)
    losses = []
    for i in range(40):
        x, y = data.batch(i, 256)
        losses.append(fused.forward_backward(x, y).item())
        opt.step()
    assert sum(losses[-5:]) / 5 < losses[0] * 0.7, losses


def test_optimizer_step_survives_graph_replays(gpu, tmp_path):
    """The optimizer's device step counter advances on every hipGraph replay (and in the fused CNN update);
    state_dict() -- hence a snapshot's OPTIMIZER_STATE -- reports it, and a reload resumes from it."""
    from pytorch_distributed_examples_amd.elastic.snapshot import load_snapshot, save_snapshot
    from pytorch_distributed_examples_amd.models.cnn import Net
    from pytorch_distributed_examples_amd.models.cnn_fused import FusedCNN
    from pytorch_distributed_examples_amd.ops.optim import FusedAdam, FusedSGD

    torch.manual_seed(0)
    lin = torch.nn.Linear(16, 4).to(gpu)
    opt = FusedAdam(lin.parameters(), lr=1e-3)
    for p in lin.parameters():
        p.grad = torch.ones_like(p)
    opt.step()                                   # eager: step 1
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        opt.step()                               # warm-up on the side stream: step 2
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        opt.step()                               # captured (not executed)
    for _ in range(5):
        g.replay()                               # steps 3..7
    torch.cuda.synchronize()
    sd = opt.state_dict()
    assert all(st["step"] == 7 for st in sd["state"].values()), sd["state"]
    path = str(tmp_path / "snap.pt")
    save_snapshot(path, lin.state_dict(), 3, sd)
    opt2 = FusedAdam(lin.parameters(), lr=1e-3)
    opt2.load_state_dict(load_snapshot(path)["OPTIMIZER_STATE"])
    opt2.step()
    assert all(st["step"] == 8 for st in opt2.state_dict()["state"].values())
    # fused CNN update paths advance the same counter
    net = Net().to(gpu).train()
    sgd = FusedSGD(net.parameters(), lr=0.01)
    f = FusedCNN(net)
    x = torch.randn(64, 1, 28, 28, device=gpu)
    y = torch.randint(0, 10, (64,), device=gpu)
    buf = f.grad_buffer()
    f.forward_backward(x, y, grad_out=buf, sgd=sgd)   # update inside the reduction
    f.forward_backward(x, y, grad_out=buf)
    f.sgd_step(sgd, buf)                               # separate update launch
    torch.cuda.synchronize()
    assert all(st["step"] == 2 for st in sgd.state_dict()["state"].values())


def test_fused_cnn_training_is_visible_to_eval(gpu):
    """After fused training steps (update inside the slab reduction), the layer-by-layer eval forward sees
    the updated weights: it matches a forward through a fresh copy of the same state_dict."""
    from pytorch_distributed_examples_amd.models.cnn import Net
    from pytorch_distributed_examples_amd.models.cnn_fused import FusedCNN
    from pytorch_distributed_examples_amd.ops.optim import FusedSGD

    torch.manual_seed(0)
    net = Net().to(gpu).train()
    sgd = FusedSGD(net.parameters(), lr=0.5)
    f = FusedCNN(net)
    x = torch.randn(256, 1, 28, 28, device=gpu)
    y = torch.randint(0, 10, (256,), device=gpu)
    net.eval()
    before = net(x).float()
    net.train()
    buf = f.grad_buffer()
    for _ in range(3):
        f.forward_backward(x, y, grad_out=buf, sgd=sgd)
    net.eval()
    after = net(x).float()
    fresh = Net().to(gpu).eval()
    fresh.load_state_dict(net.state_dict())
    ref = fresh(x).float()
    assert (after - before).abs().max().item() > 1e-3  # the weights moved
    assert torch.allclose(after, ref, atol=2e-2, rtol=2e-2)


def test_fused_mlp_folded_adam_matches_separate_step(gpu):
    """FusedMLP.forward_backward(opt=...) folds each layer's Adam update into the next backward GEMM launch
    (optimiser blocks appended to the paired dgrad + wgrad grid, layers 0-1 in a closing launch).  Same
    device update code as the separate multi-tensor step: weights, Adam moments, bf16 compute copies and the
    device step counter must match the unfused schedule after several steps (to an ulp-level drift)."""
    from pytorch_distributed_examples_amd.models.mlp import reference_mlp
    from pytorch_distributed_examples_amd.models.mlp_fused import FusedMLP
    from pytorch_distributed_examples_amd.ops.optim import FusedAdam

    torch.manual_seed(0)
    base = reference_mlp()
    g = torch.Generator().manual_seed(1)
    xs = [torch.randn(128, 1, 28, 28, generator=g).to(gpu) for _ in range(4)]
    ys = [torch.randint(0, 10, (128,), generator=g).to(gpu) for _ in range(4)]
    runs = []
    for fold in (False, True):
        net = copy.deepcopy(base).to(gpu)
        opt = FusedAdam(net.parameters(), lr=1e-3)
        f = FusedMLP(net)
        losses = []
        for x, y in zip(xs, ys):
            if fold:
                loss = f.forward_backward(x, y, opt=opt)
            else:
                loss = f.forward_backward(x, y)
                opt.step()
            losses.append(float(loss))
        torch.cuda.synchronize()
        st = opt.state_dict()
        flat = torch.cat([p.detach().reshape(-1) for p in net.parameters()])
        moments = torch.cat([opt.state[p]["exp_avg_sq"].reshape(-1) for p in net.parameters()])
        copies = torch.cat([OF._bf16_weight(L.weight).float().reshape(-1) for L in f.layers])
        runs.append((losses, flat, moments, copies, st["state"][0]["step"]))
    (l0, f0, m0, c0, s0), (l1, f1, m1, c1, s1) = runs
    assert s0 == s1 == 4, (s0, s1)
    # same device code, but compiled into two kernels: the compiler's FMA contraction differs by an ulp in a few
    # elements (scripts/diag_fold_opt.py: 1e-9 after one step), which later steps' gradients carry along
    assert all(abs(a - b) <= 1e-5 * abs(b) for a, b in zip(l0, l1)), (l0, l1)
    assert rel_err(f1, f0) < 1e-5 and rel_err(m1, m0) < 1e-3 and rel_err(c1, c0) < 1e-3


def test_fused_cnn_single_launch_tail_matches_two_launches(gpu, monkeypatch):
    """PDE_CNN_FUSED_TAIL=1 (single process): k_cnn_train runs the slab reduction, the fc1 weight-gradient tiles,
    the loss and the SGD + fragment refresh itself after a grid barrier -- one launch per step.  Same reduction
    code in the same order as k_cnn_reduce: losses, gradients, weights and the dropout stream (training mode)
    must match the two-launch step bit for bit over several steps, and the barrier must never time out."""
    from pytorch_distributed_examples_amd import _native
    from pytorch_distributed_examples_amd.models.cnn_fused import FusedCNN
    from pytorch_distributed_examples_amd.ops.optim import FusedSGD

    torch.manual_seed(0)
    base = Net().to(gpu).train()
    x = torch.randn(4, 1024, 1, 28, 28, device=gpu)
    y = torch.randint(0, 10, (4, 1024), device=gpu)
    runs = []
    rng = OF._rng_counter(x.device)
    rng0 = rng.clone()
    for tail in ("0", "1"):
        monkeypatch.setenv("PDE_CNN_FUSED_TAIL", tail)
        rng.copy_(rng0)  # the same dropout stream for both runs
        m = copy.deepcopy(base)
        f = FusedCNN(m)
        g = f.grad_buffer()
        opt = FusedSGD(m.parameters(), lr=0.05)
        losses = [f.forward_backward(x[i], y[i], grad_out=g, sgd=opt).item() for i in range(4)]
        torch.cuda.synchronize()
        runs.append((losses, g.clone(), f.flat.clone()))
    assert _native.C().cnn_tail_error(True) == 0
    (l0, g0, w0), (l1, g1, w1) = runs
    assert l0 == l1, (l0, l1)
    assert torch.equal(g0, g1) and torch.equal(w0, w1)


def test_fused_cnn_adamw_step_matches_multi_tensor_adamw(gpu):
    """FusedCNN.adamw_step (k_cnn_adamw: AdamW over the flat parameters + fragment refresh in ONE launch, the
    Horovod-elastic step) against (a) an fp32 torch.optim.AdamW step on the same flat gradient, every step, and
    (b) the multi-tensor FusedAdamW launch + the fragment prep over several steps: same losses, weights and optimiser
    state to fp32 rounding (the two kernels inline the same update function; the compiler may contract its
    multiply-adds differently), step counts equal, the state visible in state_dict (eval mode: no dropout)."""
    from pytorch_distributed_examples_amd.models.cnn_fused import FusedCNN
    from pytorch_distributed_examples_amd.ops import functional as OF
    from pytorch_distributed_examples_amd.ops.optim import FusedAdamW

    torch.manual_seed(0)
    m_ref = Net().to(gpu).eval()
    m_fus = copy.deepcopy(m_ref).eval()
    f_ref, f_fus = FusedCNN(m_ref), FusedCNN(m_fus)
    f_ref.always_prep = True
    o_ref = FusedAdamW(m_ref.parameters(), lr=0.01, weight_decay=0.01)
    o_fus = FusedAdamW(m_fus.parameters(), lr=0.01, weight_decay=0.01)
    g_ref, g_fus = f_ref.grad_buffer(), f_fus.grad_buffer()
    p_t = f_fus.flat.detach().clone().requires_grad_(True)
    o_t = torch.optim.AdamW([p_t], lr=0.01, weight_decay=0.01)
    gen = torch.Generator().manual_seed(3)
    batches = [(torch.randn(128, 1, 28, 28, generator=gen).to(gpu), torch.randint(0, 10, (128,), generator=gen).to(gpu))
               for _ in range(4)]
    ref_losses = []
    for x, y in batches:  # the reference run first: its optimiser steps bump the global weight generation
        ref_losses.append(f_ref.forward_backward(x, y, grad_out=g_ref).clone())
        o_ref.step()
    for i, (x, y) in enumerate(batches):  # then the fused run: its 2nd..4th steps reuse k_cnn_adamw's fragments
        l_fus = f_fus.forward_backward(x, y, grad_out=g_fus)
        if i > 0:
            assert f_fus._frag_gen == OF.weight_generation()  # no prep launch: the fragments come from k_cnn_adamw
        with torch.no_grad():
            p_t.copy_(f_fus.flat)
        p_t.grad = g_fus.detach().clone()
        f_fus.adamw_step(o_fus, g_fus)
        o_t.step()
        torch.cuda.synchronize()
        torch.testing.assert_close(f_fus.flat, p_t.detach(), rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(l_fus, ref_losses[i], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(f_ref.flat, f_fus.flat, rtol=1e-5, atol=1e-6)
    sa, sb = o_ref.state_dict()["state"], o_fus.state_dict()["state"]
    assert len(sa) == len(sb) == 8
    for k in sa:
        torch.testing.assert_close(sa[k]["exp_avg"], sb[k]["exp_avg"], rtol=1e-5, atol=1e-7)
        torch.testing.assert_close(sa[k]["exp_avg_sq"], sb[k]["exp_avg_sq"], rtol=1e-5, atol=1e-9)
        assert int(sa[k]["step"]) == int(sb[k]["step"]) == 4


@pytest.mark.parametrize("grouped", [1, 2])
def test_bottleneck_backward_dgrad_slabs_into_batchnorm(gpu, grouped):
    """conv2 / conv3 dgrads of a Bottleneck (inputs: bn1 / bn2 + ReLU outputs, consumed by that conv alone,
    ``dx_bn``) leave their split-K slabs unreduced and the BatchNorm backward sums them itself: at the stage-2
    micro-batch (layer3 / layer4, 8 images; grouped BatchNorm too) the block's input and parameter gradients match
    the path with the dgrads' own reduce launches (PDE_BN_BWD_DEFER=0) to bf16 rounding, the BatchNorm backward
    really took slabs, and no deferred output is left behind."""
    C = OF._C()
    torch.manual_seed(5)
    s2 = ResNetShard2()
    for blk, (c, hw) in ((s2.seq[0][1], (1024, 8)), (s2.seq[1][1], (2048, 4))):
        x = torch.randn(8, hw, hw, c).to(torch.bfloat16).to(gpu)
        gen = torch.Generator().manual_seed(c)
        outs = []
        for defer in (True, False):
            OF._BN_BWD_DEFER[0] = defer
            try:
                b = copy.deepcopy(blk).to(gpu).train()
                for it in range(2):  # the 2nd backward has .grad sinks: dgrad + wgrad paired (the deferring path)
                    for p in b.parameters():
                        if p.grad is not None:
                            p.grad.zero_()
                    xg = x.clone().requires_grad_()
                    before = C.bn_bwd_slab_uses()
                    with OF.bn_groups(grouped):
                        y = b(xg)
                    gy = torch.randn(y.shape, generator=gen.manual_seed(c)).to(torch.bfloat16).to(gpu)
                    y.backward(gy)
                    torch.cuda.synchronize()
                    used = C.bn_bwd_slab_uses() - before
            finally:
                OF._BN_BWD_DEFER[0] = True
            assert C.pending_conv_count() == 0
            grads = torch.cat([p.grad.float().reshape(-1) for p in b.parameters()])
            outs.append((xg.grad.float(), grads, used))
        (da, ga, ua), (db, gb, ub) = outs
        assert ua >= 1 and ub == 0, (c, ua, ub)
        assert rel_err(da, db) < 2e-2, (c, rel_err(da, db))
        assert rel_err(ga, gb) < 2e-2, (c, rel_err(ga, gb))
    OF.check_device_errors("dgrad slabs into bn_bwd")
