"""Fused training step for the MNIST CNN (csrc/kernels/cnn_fused.hip).

:class:`FusedCNN` flattens a :class:`~.cnn.Net`'s parameters into ONE contiguous fp32 buffer in torch
parameter order (the ``nn.Parameter`` objects stay the same, their storage becomes views of the flat
buffer, so optimizers / ``state_dict`` / DDP keep working) and runs forward + NLL + backward of the
whole batch in one kernel launch plus one deterministic slab-reduction that writes the gradients
straight into a flat gradient buffer -- the DDP wrapper's, when it is laid out in forward order.

    fused = FusedCNN(net)
    ddp = DistributedDataParallel(net, overlap=False, param_order="forward")
    loss = fused.forward_backward(x, y, grad_out=ddp.flat_grad)   # grads written, no autograd
    ddp.sync_gradients(); opt.step()

Semantics match ``nll_loss(net(x), y)`` + ``backward()`` in train mode, including Dropout2d(p=0.5) on
conv2's output and dropout(p=0.5) on fc1's (fresh masks every call; dropout disabled in eval mode).
"""
from __future__ import annotations

import torch

from .. import _native
from ..ops import functional as OF


class FusedCNN:
    def __init__(self, net, workgroups: int | None = None):
        C = _native.C()
        self.net = net
        self.params = list(net.parameters())
        n = sum(p.numel() for p in self.params)
        assert n == C.cnn_num_params(), f"not the reference Net ({n} params)"
        dev = self.params[0].device
        flat = torch.empty(n, dtype=torch.float32, device=dev)
        off = 0
        with torch.no_grad():
            for p in self.params:
                k = p.numel()
                flat[off:off + k].copy_(p.detach().reshape(-1))
                p.data = flat[off:off + k].view_as(p)
                off += k
        self.flat = flat
        self.own_grad = None
        self.workgroups = workgroups
        self.stamps = None  # diagnostic: int64 [nwg, 16] tensor of per-phase wall-clock stamps

    def _nwg(self, B: int) -> int:
        if self.workgroups:
            return self.workgroups
        # ~4 images per workgroup, one workgroup per CU (256 CUs); 2 fit per CU by LDS
        return max(1, min(512, (B + 3) // 4))

    def grad_buffer(self) -> torch.Tensor:
        """A flat gradient buffer whose views are installed as ``p.grad`` (when no DDP buffer is used)."""
        if self.own_grad is None:
            self.own_grad = torch.zeros_like(self.flat)
            off = 0
            for p in self.params:
                k = p.numel()
                p.grad = self.own_grad[off:off + k].view_as(p)
                off += k
        return self.own_grad

    def forward_backward(self, x: torch.Tensor, y: torch.Tensor, grad_out: torch.Tensor | None = None,
                         accumulate: bool = False, p_drop2: float = 0.5, p_drop1: float = 0.5) -> torch.Tensor:
        """Loss (device scalar) of the batch; gradients of the mean loss written to ``grad_out``."""
        C = _native.C()
        if grad_out is None:
            grad_out = self.grad_buffer()
        x = x.float().contiguous()
        y = y.long().contiguous()
        training = self.net.training
        loss = C.cnn_train(x, y, self.flat, OF._rng_counter(x.device), p_drop2, p_drop1, training, grad_out,
                           accumulate, None, self.stamps)
        OF.bump_weight_generation()
        return loss
