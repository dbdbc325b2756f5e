"""GPU training step of the Horovod MNIST CNN scripts with ANY wrapped optimiser (horovod_mnist_elastic.py uses
AdamW, :41-42), captured into a hipGraph.

    step = FusedHvdStep(model, optimizer, batch)   # optimizer = hvd.DistributedOptimizer(FusedAdamW(...))
    loss = step(x, y)                              # forward + backward + all-reduce + AdamW
    step.reset()                                   # after an elastic reset (new engine / world size)

* forward + backward: the whole-network fused kernel (:class:`..models.cnn_fused.FusedCNN`), gradients written
  into ``p.grad`` views of ONE flat buffer -- so the fusion engine reduces the batch in place (one xGMI one-shot
  exchange, no pack / unpack) -- with the bf16 weight-fragment image rebuilt from the fp32 weights inside the
  kernel every step (``always_prep``: the optimiser is not the fused SGD);
* ``optimizer.step()``: ``synchronize()`` (the engine; in graph mode stream-ordered on the caller's stream) then the
  wrapped multi-tensor optimiser (FusedAdamW: hyper-parameters and step count in device memory);
* the first call after construction or :meth:`reset` runs eagerly through the engine -- it negotiates the gradient
  names into the response cache -- then ``enable_graph_mode`` and the step is captured: every later full-batch call
  is ONE graph replay (the batch copied into the graph's static slots).  A short last batch runs eagerly.
  :meth:`reset` drops the graph (the xGMI view, the world size and the learning rate are baked into it).
"""
from __future__ import annotations

import torch

from ..models.cnn_fused import FusedCNN


class FusedHvdStep:
    def __init__(self, model, optimizer, batch: int, graph: bool = True):
        self.model, self.opt, self.batch = model, optimizer, int(batch)
        self.fused = FusedCNN(model)
        from ..ops.optim import FusedSGD

        # plain FusedSGD (the DP script, mnist_horovod.py:50): the update rides in the fused kernel's slab reduction
        # at world 1, else ONE launch after the engine's synchronize that also refreshes the bf16 fragment image --
        # the bench's hvd_cnn step.  Other optimisers (AdamW): the multi-tensor update, fragments rebuilt in-kernel.
        from ..ops.optim import FusedAdamW

        g = optimizer.param_groups[0] if len(optimizer.param_groups) == 1 else None
        self.sgd_fast = (isinstance(optimizer, FusedSGD) and g is not None and g.get("momentum", 0.0) == 0.0
                         and g.get("weight_decay", 0.0) == 0.0)
        # one-group FusedAdamW (the elastic script): update + fragment refresh in ONE launch (FusedCNN.adamw_step)
        self.adamw_fast = isinstance(optimizer, FusedAdamW) and g is not None
        self.fused.always_prep = not (self.sgd_fast or self.adamw_fast)
        if not self.sgd_fast:
            from ..ops import functional as OF

            # the kernel rebuilds its fragment image from the fp32 weights every step: the optimiser need not keep
            # the layer path's bf16 conv / linear layouts current (an eager model(x) falls back to cached copies)
            for p in model.parameters():
                p.__dict__["_pde_own_copies"] = True
                OF.release_compute_copies(p)
        self.grads = self.fused.grad_buffer()  # p.grad: views of one flat buffer (never set to None)
        self.use_graph = graph
        self.graph = None
        self.negotiated = False
        self.replays = 0

    def _eager(self, x, y):
        if self.sgd_fast:
            from . import core

            if core.size() == 1:  # all-reduce = identity: SGD inside the reduction kernel
                self.opt.synchronize()
                return self.fused.forward_backward(x, y, grad_out=self.grads, sgd=self.opt)
            loss = self.fused.forward_backward(x, y, grad_out=self.grads)
            self.opt.synchronize()  # the engine (graph mode: stream-ordered on this stream)
            with self.opt.skip_synchronize():
                self.fused.sgd_step(self.opt, self.grads)
            return loss
        loss = self.fused.forward_backward(x, y, grad_out=self.grads)
        if self.adamw_fast:
            self.opt.synchronize()  # the engine (graph mode: stream-ordered on this stream)
            with self.opt.skip_synchronize():
                self.fused.adamw_step(self.opt, self.grads)
            return loss
        self.opt.step()
        return loss

    def eager_step(self, x, y):
        """One eager step; the first one negotiates through the engine and turns graph mode on, so every later call
        is capturable (an epoch-graph runner, utils/epoch_graph.py, captures this function)."""
        loss = self._eager(x, y)
        if not self.negotiated:
            torch.cuda.synchronize()
            self.opt.enable_graph_mode()
            self.negotiated = True
        return loss

    def __call__(self, x, y):
        if not self.use_graph or x.shape[0] != self.batch:
            return self._eager(x, y)
        if self.graph is None:
            if not self.negotiated:  # one step through the engine: every gradient enters the response cache
                loss = self._eager(x, y)
                torch.cuda.synchronize()
                self.opt.enable_graph_mode()
                self.negotiated = True
                return loss
            from ..utils.graph import CapturedStep

            # no warm-up steps: the negotiated eager step already initialised everything (a warm-up would train
            # one extra step on this batch)
            self.graph = CapturedStep(self._eager, [x, y], warmup=0).capture()
        self.replays += 1
        return self.graph(x, y)

    def reset(self):
        """After an elastic reset: drop the graph and negotiate again through the new engine."""
        self.graph = None
        self.negotiated = False
        if hasattr(self.opt, "disable_graph_mode"):
            self.opt.disable_graph_mode()
        self.fused.invalidate()
