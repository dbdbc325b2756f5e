"""``hvd.DistributedOptimizer`` and gradient compression (horovod/torch/optimizer.py semantics).

Used by the reference at horovod/mnist_horovod.py:53 and horovod/horovod_mnist_elastic.py:42.

* A post-accumulate-grad hook per parameter enqueues an asynchronous in-place all-reduce of ``p.grad``
  on the C++ fusion engine as soon as the gradient is final (after ``backward_passes_per_step`` passes),
  so communication overlaps the rest of backward; the engine fuses them into xGMI-sized buffers.
* ``step()`` synchronizes (waits every handle; GPU: stream-ordered, no host block) then runs the wrapped
  optimizer's step -- works with torch optimizers and with the fused multi-tensor optimizers of
  :mod:`..ops.optim`.
* ``op=Average`` uses RCCL's in-collective average (no extra kernel); ``gradient_predivide_factor``
  splits the averaging into a pre-scale in the pack kernel and a post-scale in the unpack kernel.
* Graph mode (:meth:`enable_graph_mode`, MI355X addition): once the engine's response cache holds every
  parameter (one step negotiated through the engine), ``synchronize()`` enqueues the same fused batches on
  the caller's stream -- no engine thread, no host wait -- so the whole training step records into a hipGraph.
  SPMD: every rank must reach ``synchronize()`` each step (as with a captured DDP step).
* ``Compression.fp16`` sends fp32 gradients as bf16 on the wire (CDNA4's native 16-bit training format;
  same bytes as fp16, fp32 exponent range); ``Compression.bf16`` is the explicit name.
"""
from __future__ import annotations

import contextlib

import torch

from . import core
from ..ops import streams
from .exceptions import HorovodInternalError


class _NoneCompressor:
    wire_bf16 = False

    @staticmethod
    def compress(tensor):
        return tensor, None

    @staticmethod
    def decompress(tensor, ctx):
        return tensor


class _BF16Compressor:
    wire_bf16 = True

    @staticmethod
    def compress(tensor):
        if tensor.dtype.is_floating_point and tensor.dtype != torch.bfloat16:
            return tensor.to(torch.bfloat16), tensor.dtype
        return tensor, None

    @staticmethod
    def decompress(tensor, ctx):
        return tensor.to(ctx) if ctx is not None else tensor


class Compression:
    none = _NoneCompressor
    fp16 = _BF16Compressor
    bf16 = _BF16Compressor


class _DistributedOptimizerMixin:
    def _hvd_setup(self, named_parameters, compression, backward_passes_per_step, op, gradient_predivide_factor):
        self._compression = compression
        self._op = op
        self._bpps = backward_passes_per_step
        self._predivide = gradient_predivide_factor
        if named_parameters is not None:
            named = list(named_parameters)
        else:
            named = [(f"allreduce.noname.{i}.{j}", p) for i, g in enumerate(self.param_groups)
                     for j, p in enumerate(g["params"])]
        names = [n for n, _ in named]
        if len(set(names)) != len(names):
            raise ValueError("Parameter names in named_parameters must be unique.")
        all_params = {id(p) for g in self.param_groups for p in g["params"]}
        missing = [p for p in all_params if p not in {id(q) for _, q in named}]
        if missing:
            raise ValueError("named_parameters was specified, but one or more model parameters were not named.")
        self._param_names = {p: n for n, p in named}
        self._handles: dict = {}
        self._counts = {p: 0 for _, p in named}
        self._synchronized = False
        self._should_sync = True
        self._graph = False
        self._hooks = []
        if core.size() > 1:
            for _, p in named:
                if p.requires_grad:
                    self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook()))

    def _make_hook(self):
        def hook(p):
            if self._graph:  # graph mode: reduced in synchronize(), stream-ordered
                return
            if p in self._handles and self._handles[p] is not None:
                # the gradient was already handed to the engine (in-place all-reduce in flight): another
                # local pass would race with it and mix reduced and unreduced values
                raise AssertionError("Gradients were computed more than backward_passes_per_step times "
                                     "before call to step(). Increase backward_passes_per_step to "
                                     "accumulate gradients locally.")
            self._counts[p] += 1
            if self._counts[p] >= self._bpps:
                self._handles[p] = self._allreduce_grad(p)
                self._counts[p] = 0

        return hook

    def _allreduce_grad(self, p):
        name = self._param_names.get(p)
        g = p.grad
        if g.is_cuda:  # the gradient may still be in flight on the wgrad side stream (ops/streams.py)
            streams.join(g.device)
        if not g.is_contiguous():
            p.grad = g = g.contiguous()
        op = self._op
        pre, post = 1.0, 1.0
        if self._predivide != 1.0 and op == core.ReduceOp.Average:
            # sum with pre/post scaling: result = sum(g / f) * (f / size)
            op = core.ReduceOp.Sum
            pre, post = 1.0 / self._predivide, self._predivide / core.size()
        # (like Horovod, locally accumulated passes are summed, not averaged, before the all-reduce)
        return core.allreduce_async_(g, name=name, op=op, prescale_factor=pre, postscale_factor=post,
                                     compression_bf16=self._compression.wire_bf16)

    def enable_graph_mode(self):
        """Reduce gradients stream-ordered (hipGraph-capturable) from now on.  Needs every parameter's
        all-reduce in the response cache, i.e. at least one step synchronized through the engine."""
        if core.size() > 1:
            missing = [n for n in self._param_names.values() if not core.is_cached(n)]
            if missing:
                raise RuntimeError(f"graph mode needs a negotiated step first; not cached: {missing[:4]}")
            # size the engine's inline staging buffer for this gradient set now (never while capturing) and
            # park its idle negotiation loop: replays bypass it (health: core.check_health at commits)
            core.set_graph_mode(True, [p.grad if p.grad is not None else p for p in self._param_names])
        self._graph = True
        return self

    def disable_graph_mode(self):
        if self._graph and core.size() > 1:
            core.set_graph_mode(False)
        self._graph = False
        return self

    def _graph_synchronize(self):
        op, pre, post = self._op, 1.0, 1.0
        if self._predivide != 1.0 and op == core.ReduceOp.Average:
            op, pre, post = core.ReduceOp.Sum, 1.0 / self._predivide, self._predivide / core.size()
        grads = [p.grad for p in self._param_names if p.grad is not None]
        if grads and grads[0].is_cuda:
            streams.join(grads[0].device)
        core.allreduce_inline_(grads, op, pre, post, self._compression.wire_bf16)
        for p in self._param_names:
            self._counts[p] = 0
        self._synchronized = True

    def synchronize(self):
        if core.size() == 1:
            self._synchronized = True
            return
        if self._graph:
            return self._graph_synchronize()
        # parameters whose gradient was produced but whose hook count did not reach bpps, or that got no
        # gradient at all this step, are reduced now (same order on every rank: registration order)
        for p in self._param_names:
            if p not in self._handles or self._handles[p] is None:
                if p.grad is not None:
                    self._handles[p] = self._allreduce_grad(p)
            # every parameter starts the next accumulation window from zero passes (Horovod resets the
            # delay of every handled parameter), including those reduced early here
            self._counts[p] = 0
        try:
            for p, h in list(self._handles.items()):
                if h is not None:
                    core.synchronize(h)
        except HorovodInternalError:
            self._handles.clear()
            raise
        self._handles.clear()
        self._synchronized = True

    @contextlib.contextmanager
    def skip_synchronize(self):
        self._should_sync = False
        try:
            yield
        finally:
            self._should_sync = True

    def step(self, closure=None):
        if self._should_sync:
            if self._synchronized:
                pass
            else:
                self.synchronize()
        self._synchronized = False
        return super().step(closure)  # type: ignore[misc]

    def zero_grad(self, set_to_none: bool = True):
        if any(h is not None for h in self._handles.values()):
            raise AssertionError("optimizer.zero_grad() was called after loss.backward() but before "
                                 "optimizer.step() or optimizer.synchronize().")
        return super().zero_grad(set_to_none=set_to_none)  # type: ignore[misc]


def DistributedOptimizer(optimizer, named_parameters=None, compression=Compression.none,
                         backward_passes_per_step: int = 1, op=core.ReduceOp.Average,
                         gradient_predivide_factor: float = 1.0, groups=None, sparse_as_dense=False):
    """Wrap ``optimizer`` so gradients are all-reduced across workers before ``step()``."""
    cls = type(optimizer.__class__.__name__, (_DistributedOptimizerMixin, optimizer.__class__), {})
    obj = cls.__new__(cls)
    obj.__dict__.update(optimizer.__dict__)
    obj._hvd_setup(named_parameters, compression, backward_passes_per_step, op, gradient_predivide_factor)
    return obj
