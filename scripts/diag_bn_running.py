"""Diagnostic: running-statistics update count of the GPU BatchNorm paths (one forward of a fresh module)."""
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from pytorch_distributed_examples_amd.ops import layers as L
from pytorch_distributed_examples_amd.ops import functional as OF
from pytorch_distributed_examples_amd.models.resnet import Bottleneck

dev = torch.device("cuda:0")
torch.manual_seed(0)
for C, P in ((64, 4096), (256, 8192), (512, 512)):
    bn = L.BatchNorm2d(C).to(dev)
    x = (torch.randn(P // 64, 8, 8, C) * 2 + 3).to(torch.bfloat16).to(dev)
    y = bn(x, relu=True)
    torch.cuda.synchronize()
    m = x.float().reshape(-1, C).mean(0)
    print(f"plain bn C={C} P={P}: running_mean/true_mean = {(bn.running_mean / m).mean().item():.4f} (expect 0.1)")
for fold in (True, False):
    OF._BN_FOLD[0] = fold
    torch.manual_seed(1)
    blk = Bottleneck(256, 64)
    x = torch.randn(8, 256, 32, 32).to(torch.bfloat16).float()
    ref = blk(x)
    g = copy.deepcopy(Bottleneck(256, 64)).to(dev)
    g.load_state_dict(Bottleneck(256, 64).state_dict()) if False else None
    g = copy.deepcopy(blk)
    # reset blk's stats copy on g
    for n, b in g.named_buffers():
        if "running_mean" in n: b.zero_()
        if "running_var" in n: b.fill_(1.0)
    g = g.to(dev)
    out = g(x.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).to(dev))
    torch.cuda.synchronize()
    for n in ("bn1", "bn2", "bn3"):
        ra = getattr(g, n).running_mean.cpu()
        rb = getattr(blk, n).running_mean
        print(f"fold={fold} {n}: gpu/cpu running_mean ratio {(ra.norm() / rb.norm()).item():.4f}")
