"""Diagnostic: FusedMLP with the Adam update folded into the backward launches vs the separate step -- per
step and per layer, the max |difference| of the weights (GPU)."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_examples_amd.models.mlp import reference_mlp  # noqa: E402
from pytorch_distributed_examples_amd.models.mlp_fused import FusedMLP  # noqa: E402
from pytorch_distributed_examples_amd.ops.optim import FusedAdam  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
base = reference_mlp()
g = torch.Generator().manual_seed(1)
xs = [torch.randn(128, 1, 28, 28, generator=g).to(dev) for _ in range(4)]
ys = [torch.randint(0, 10, (128,), generator=g).to(dev) for _ in range(4)]
nets, opts, fs = [], [], []
for fold in (False, True):
    net = copy.deepcopy(base).to(dev)
    nets.append(net)
    opts.append(FusedAdam(net.parameters(), lr=1e-3))
    fs.append(FusedMLP(net))
for step, (x, y) in enumerate(zip(xs, ys)):
    la = fs[0].forward_backward(x, y)
    ga = [p.grad.clone() for p in nets[0].parameters()]
    opts[0].step()
    lb = fs[1].forward_backward(x, y, opt=opts[1])
    gb = [p.grad.clone() for p in nets[1].parameters()]
    torch.cuda.synchronize()
    print(f"step {step}: loss {float(la):.6f} {float(lb):.6f}")
    for k, (pa, pb, a, b) in enumerate(zip(nets[0].parameters(), nets[1].parameters(), ga, gb)):
        dp = (pa - pb).abs().max().item()
        dg = (a - b).abs().max().item()
        if dp or dg:
            print(f"  param {k} {tuple(pa.shape)}: max|dW| {dp:.3e} max|dgrad| {dg:.3e}")
