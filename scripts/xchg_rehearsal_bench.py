"""Rehearsal timing of the fused CNN's world > 1 step on ONE GPU: 2 processes share the card (gloo control
plane, peers mapped over IPC exactly as on a node).  Compares, per step of 1024 images per rank:

  xchg   forward_backward(..., sgd, xgmi)      2 launches (exchange + SGD inside the reduction kernel)
  3step  forward_backward + xGMI all-reduce kernel + SGD launch   (PDE_CNN_XCHG=0 path)
  local  forward_backward(..., sgd) without any exchange          (lower bound: world-1 work)

Both processes run the same loop at the same time, so every number includes sharing the GPU with the
other rank's kernels; the differences between the modes are the exchange's cost.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 scripts/xchg_rehearsal_bench.py
"""
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("PDE_BACKEND", "gloo")

from pytorch_distributed_examples_amd.models.cnn import Net  # noqa: E402
from pytorch_distributed_examples_amd.models.cnn_fused import FusedCNN  # noqa: E402
from pytorch_distributed_examples_amd.ops.optim import FusedSGD  # noqa: E402
from pytorch_distributed_examples_amd.parallel import dist as pdist  # noqa: E402
from pytorch_distributed_examples_amd.parallel.xgmi_allreduce import XgmiAllreduce  # noqa: E402

ctx = pdist.init_distributed()
dev, r, N = ctx.device, ctx.rank, ctx.world_size
torch.manual_seed(0)
net = Net().to(dev)
fused = FusedCNN(net)
opt = FusedSGD(net.parameters(), lr=0.01)
g = fused.grad_buffer()
xa = XgmiAllreduce(dev, timeout_s=20.0)
B = int(os.environ.get("XB", "1024"))
x = torch.randn(B, 1, 28, 28, device=dev)
y = torch.randint(0, 10, (B,), device=dev)


def step_xchg():
    fused.forward_backward(x, y, grad_out=g, sgd=opt, xgmi=xa)


def step_3():
    fused.forward_backward(x, y, grad_out=g)
    xa.allreduce_(g, avg=True)
    fused.sgd_step(opt, g)


def step_local():
    fused.forward_backward(x, y, grad_out=g, sgd=opt)


res = {}
iters = int(os.environ.get("XITERS", "300"))
for name, fn in (("xchg", step_xchg), ("3step", step_3), ("local", step_local), ("xchg_again", step_xchg)):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    dist.barrier()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(iters):
        fn()
    t1.record()
    torch.cuda.synchronize()
    res[name] = round(t0.elapsed_time(t1) * 1000.0 / iters, 2)
    dist.barrier()
xa.check()
out = [None] * N
dist.all_gather_object(out, res)
if r == 0:
    print(json.dumps({"us_per_step_per_rank": out, "batch_per_rank": B, "ranks_sharing_one_gpu": N}))
xa.close()
dist.destroy_process_group()
