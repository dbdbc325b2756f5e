"""Weight-gradient side stream: backward GEMMs that are off the critical path run concurrently.

In a layer's backward the data gradient (dgrad) feeds the previous layer, the weight gradient (wgrad) feeds
only the optimizer (and the gradient all-reduce).  At the reference's small per-GPU batches the GEMMs are
latency-bound (ResNet-50 at batch 32: layer4's convolutions have 512 output rows; the MLP at batch 128), so
one stream leaves most of the 256 CUs idle between dependent launches.  Here every wgrad of a conv / linear
layer is issued on a per-device side stream, forked from the producing stream right after the layer's
output gradient exists; the dgrad chain keeps the main stream.  Inside a captured hipGraph the fork / join
become graph edges, so the two chains run as parallel branches of one replay.

Joins (the main stream waits for every wgrad issued so far):

* at the end of each autograd backward pass (an engine final callback, onto the stream the layer's backward
  ran on -- the forward stream);
* before any reader of ``.grad`` that may run earlier: DDP bucket launches (overlapped hooks and
  ``sync_gradients``), the Horovod hooks, the fused optimizers;
* explicitly by launch sequences that fork themselves (:class:`..models.mlp_fused.FusedMLP`).

Tensors read on the side stream are ``record_stream``-ed so the caching allocator never recycles them under
a running wgrad.

OFF by default (``PDE_WGRAD_STREAM=1`` or :func:`set_enabled` turns it on).  Measured on one MI355X
(scripts/gpu_streams.sh, hipGraph-captured steps): ResNet-50 128px b32 4.48 -> 5.01 ms/step and the fused
MLP 0.254 -> 0.345 ms/step WITH the side stream -- a hipGraph with parallel branches is launched node by node
across hardware queues with cross-queue barrier packets at every fork / join, which costs more than the
overlap wins at these kernel sizes.  The concurrency the side stream was meant to buy is delivered instead
by pairing each layer's dgrad and wgrad into ONE launch (``gemm_pair`` in :mod:`.functional`,
``pde::gemm_bf16_pair``), which keeps the graph linear.

Reference: the dgrad / wgrad pair is what autograd computes for every ``nn.Conv2d`` / ``nn.Linear`` of
rpc/model_parallel_ResNet50.py:85-139 and pytorch_elastic/mnist_ddp_elastic.py:133-159.
"""
from __future__ import annotations

import contextlib
import os

import torch

_ENABLED = [os.environ.get("PDE_WGRAD_STREAM", "0") == "1"]
_SIDE: dict = {}      # device index -> side stream
_PENDING: dict = {}   # device index -> True while side work exists that no join has covered yet


def enabled() -> bool:
    return _ENABLED[0]


def set_enabled(flag: bool) -> None:
    _ENABLED[0] = bool(flag)


@contextlib.contextmanager
def disabled():
    old = _ENABLED[0]
    _ENABLED[0] = False
    try:
        yield
    finally:
        _ENABLED[0] = old


def side_stream(device) -> torch.cuda.Stream:
    idx = torch.device(device).index
    idx = torch.cuda.current_device() if idx is None else idx
    s = _SIDE.get(idx)
    if s is None:
        with torch.cuda.device(idx):
            s = torch.cuda.Stream(priority=0)
        _SIDE[idx] = s
    return s


@contextlib.contextmanager
def fork(*tensors, join_at_backward_end: bool = True):
    """Run the body on the side stream, ordered after everything issued so far on the current stream.
    ``tensors`` are read by the body (they are kept alive for the side stream).  ``join_at_backward_end``
    queues a join onto the current stream at the end of the running autograd backward pass."""
    dev = tensors[0].device
    origin = torch.cuda.current_stream(dev)
    side = side_stream(dev)
    side.wait_stream(origin)
    for t in tensors:
        if t is not None and t.is_cuda:
            t.record_stream(side)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    if join_at_backward_end and not _PENDING.get(idx):
        try:
            torch.autograd.Variable._execution_engine.queue_callback(lambda: _join_onto(idx, origin))
        except RuntimeError:  # not inside a backward pass: the caller joins explicitly
            pass
    _PENDING[idx] = True
    with torch.cuda.stream(side):
        yield side


def _join_onto(idx: int, stream: torch.cuda.Stream) -> None:
    if _PENDING.get(idx):
        stream.wait_stream(_SIDE[idx])
        _PENDING[idx] = False


# ---- deferred weight-gradient reductions ---------------------------------------------------------------
# The paired backward GEMMs (ops/functional.py ``gemm_pair(defer=True)``) leave the split-K slab reduction of
# their weight gradient pending; ONE batched launch reduces all of them (pde::gemm_reduce_jobs) when the
# gradients are first needed: at the end of the backward pass (engine final callback) or earlier at any
# gradient reader that joins (DDP bucket launch, Horovod hook, fused optimizer).  That replaces one reduce
# launch per layer with one per step.  ``PDE_DEFER_WGRAD_REDUCE=0`` reduces every pair right away.
_DEFER_ENABLED = [os.environ.get("PDE_DEFER_WGRAD_REDUCE", "1") != "0"]
_DEFERRED: dict = {"stream": None}


def defer_enabled() -> bool:
    return _DEFER_ENABLED[0]


def note_deferred_reduce(flush_by_caller: bool = False) -> None:
    """A weight-gradient reduction was deferred on the current stream: queue the end-of-backward flush.
    Outside a regular autograd backward pass (e.g. a distributed-autograd engine that takes no final callbacks)
    it is flushed right away, unless ``flush_by_caller`` (an explicit launch sequence that joins itself)."""
    if _DEFERRED["stream"] is None:
        _DEFERRED["stream"] = torch.cuda.current_stream()
        if flush_by_caller:
            return
        try:
            torch.autograd.Variable._execution_engine.queue_callback(flush_deferred)
        except RuntimeError:  # no backward pass to hook: never leave gradients unreduced
            flush_deferred()


def flush_deferred(stream: torch.cuda.Stream | None = None) -> None:
    """Launch the pending weight-gradient reductions (on the stream that produced them); ``stream`` then
    waits for them when it is a different stream."""
    s = _DEFERRED["stream"]
    if s is None:
        return
    _DEFERRED["stream"] = None
    from .. import _native

    with torch.cuda.stream(s):
        _native.C().gemm_flush_deferred()
    if stream is not None and stream != s:
        stream.wait_stream(s)


def join(device=None, stream: torch.cuda.Stream | None = None) -> None:
    """Make ``stream`` (default: the current stream of ``device``) see every gradient issued so far: pending
    deferred weight-gradient reductions are launched, side-stream work is waited for."""
    if _DEFERRED["stream"] is not None:
        flush_deferred(stream if stream is not None else torch.cuda.current_stream())
    if not _PENDING:
        return
    if device is None:
        for idx in list(_PENDING):
            if _PENDING[idx]:
                _join_onto(idx, stream if stream is not None else torch.cuda.current_stream(idx))
        return
    dev = torch.device(device)
    if dev.type != "cuda":
        return
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    _join_onto(idx, stream if stream is not None else torch.cuda.current_stream(dev))


def active_for(t: torch.Tensor) -> bool:
    """Whether a wgrad reading ``t`` should go to the side stream."""
    return _ENABLED[0] and t.is_cuda
