#!/usr/bin/env python3
"""Multi-tensor Adam bandwidth on one GPU: the MLP's parameter set (5.0M), with the linear weights' bf16
compute copies, with the gradients freshly rewritten before each step (as after a backward), and large sets;
effective TB/s = state bytes / kernel time (CUDA events around each optimizer step)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_examples_amd.ops.optim import FusedAdam  # noqa: E402


def run(shapes, label, bf16=False, rewrite=False):
    ps = []
    for s in shapes:
        p = torch.nn.Parameter(torch.randn(s, device="cuda"))
        if bf16 and len(s) == 2:
            p._pde_linear = True
        p.grad = torch.randn_like(p)
        ps.append(p)
    src = [torch.randn_like(p) for p in ps]
    opt = FusedAdam(ps, lr=1e-3)
    for _ in range(5):
        opt.step()
    torch.cuda.synchronize()
    n = 50
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        if rewrite:
            for p, s in zip(ps, src):
                p.grad.copy_(s)
        a.record()
        opt.step()
        b.record()
    torch.cuda.synchronize()
    us = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)[n // 2]
    numel = sum(p.numel() for p in ps)
    nb = sum(p.numel() for p in ps if bf16 and p.dim() == 2)
    byts = numel * 28 + nb * 2
    print(f"{label:36s} {numel / 1e6:7.2f}M params  {us:8.2f} us/step (median)  {byts / us / 1e6:6.2f} TB/s", flush=True)


if __name__ == "__main__":
    mlp = [(1024, 784), (1024,)] + [(1024, 1024), (1024,)] * 4 + [(10, 1024), (10,)]
    run(mlp, "mlp params")
    run(mlp, "mlp params + bf16 copies", bf16=True)
    run(mlp, "mlp + bf16 + grads rewritten", bf16=True, rewrite=True)
    run([(4096, 4096)] * 4, "4 x 16M")
