"""BatchNorm folded into the convolutions around it (csrc/kernels/gemm.hip BnStatsOut / BnFoldIn, VERDICT r3
ask 1): the producer conv's epilogue emits the batch statistics, the consumer conv applies bn + ReLU in its A
loader and writes the activation once.  Every ResNet-50 bottleneck shape, folded vs the one-launch BatchNorm
path (PDE_BN_FOLD off) on identical inputs and weights: outputs, input / parameter gradients and running
statistics agree to bf16 noise, twice in a row (the statistics buffer is zeroed by the consumer's last block),
plain and with grouped (per-micro-batch) BatchNorm.  The folded path is also checked against the fp32
reference of the whole block (torch on the same bf16 values)."""
import copy

import pytest
import torch

from pytorch_distributed_examples_amd.models.resnet import ResNetShard1, ResNetShard2
from pytorch_distributed_examples_amd.ops import functional as OF

pytestmark = pytest.mark.gpu


def rel_err(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


def _blocks():
    torch.manual_seed(5)
    s1, s2 = ResNetShard1(), ResNetShard2()
    return [(s1.seq[4][0], 64, 32), (s1.seq[4][1], 256, 32), (s1.seq[5][0], 256, 32), (s1.seq[5][1], 512, 16),
            (s2.seq[0][0], 512, 16), (s2.seq[0][1], 1024, 8), (s2.seq[1][0], 1024, 8), (s2.seq[1][1], 2048, 4)]


def _run(blk, x, gy, fold: bool, groups: int, steps: int = 2):
    prev = OF._BN_FOLD[0]
    OF._BN_FOLD[0] = fold
    try:
        b = copy.deepcopy(blk).to(x.device).train()
        outs = []
        for _ in range(steps):
            for p in b.parameters():
                p.grad = None
            xg = x.clone().requires_grad_()
            with OF.bn_groups(groups):
                y = b(xg)
            y.backward(gy)
            grads = torch.cat([p.grad.float().reshape(-1) for p in b.parameters()])
            outs.append((y.detach().float(), xg.grad.float(), grads))
        bufs = torch.cat([t.float().reshape(-1) for n, t in b.named_buffers() if "running" in n])
        plan = b.__dict__.get("_pde_fold_plan", {})
        return outs, bufs, plan
    finally:
        OF._BN_FOLD[0] = prev


@pytest.mark.parametrize("groups", [1, 2])
def test_folded_bottlenecks_match_unfolded(gpu, groups):
    torch.manual_seed(0)
    folded_any = 0
    for blk, c, hw in _blocks():
        x = torch.randn(8, hw, hw, c).to(torch.bfloat16).to(gpu)
        g = torch.Generator().manual_seed(c + hw)
        with torch.no_grad(), OF.bn_groups(groups):
            shape = copy.deepcopy(blk).to(gpu).eval()(x).shape
        gy = torch.randn(shape, generator=g).to(torch.bfloat16).to(gpu)
        fo, fb, plan = _run(blk, x, gy, True, groups)
        uo, ub, _ = _run(blk, x, gy, False, groups)
        folded_any += sum(int(f) for v in plan.values() for f in v)
        for step, ((yf, df, gf), (yu, du, gu)) in enumerate(zip(fo, uo)):
            assert rel_err(yf, yu) < 1e-2, (c, hw, step, rel_err(yf, yu))
            assert rel_err(df, du) < 3e-2, (c, hw, step, rel_err(df, du))
            assert rel_err(gf, gu) < 3e-2, (c, hw, step, rel_err(gf, gu))
        assert rel_err(fb, ub) < 1e-3, (c, hw, rel_err(fb, ub))
    assert folded_any >= 6, "the fold plan rejected (almost) every bottleneck shape"
    OF.check_device_errors("bn fold test")


def test_folded_bottleneck_matches_fp32_reference(gpu):
    """Forward of a folded bottleneck against the CPU fp32 module on the same bf16-rounded input."""
    from pytorch_distributed_examples_amd.models.resnet import Bottleneck

    torch.manual_seed(1)
    blk = Bottleneck(256, 64)
    x = torch.randn(8, 256, 32, 32).to(torch.bfloat16).float()
    g = copy.deepcopy(blk).to(gpu)  # (before the reference forward updates blk's running statistics)
    with OF.emulate_bf16_on_cpu():
        ref = blk(x)
    prev = OF._BN_FOLD[0]
    OF._BN_FOLD[0] = True  # the fold is opt-in (PDE_BN_FOLD=1)
    try:
        out = g(x.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).to(gpu))
    finally:
        OF._BN_FOLD[0] = prev
    assert any(any(v) for v in g._pde_fold_plan.values()), g._pde_fold_plan
    assert rel_err(out.float().permute(0, 3, 1, 2).cpu(), ref) < 3e-2
    for n in ("bn1", "bn2"):
        ra = getattr(g, n).running_mean.cpu()
        rb = getattr(blk, n).running_mean
        assert rel_err(ra, rb) < 2e-2, (n, rel_err(ra, rb))
        assert g.state_dict()[f"{n}.num_batches_tracked"].item() == 1  # (counted on the host, flushed lazily)
