"""Whole-training-step hipGraph capture (the MNIST nets are launch-bound).

A training step of this suite is a fixed sequence of HIP kernels: layout/cast kernels, MFMA GEMMs,
fused epilogues, BN/pool/loss kernels, the RCCL all-reduce of the flat gradient buffer and ONE fused
optimizer kernel whose hyper-parameters/step live in device memory.  :class:`CapturedStep` records that
sequence once into a ``torch.cuda.CUDAGraph`` (a hipGraph on ROCm) and replays it with a single launch
per step; the batch is copied into static input buffers before each replay.

Capture rules honoured by the ops layer:
* no host synchronisation inside the step (no ``.item()``; loss stays a device tensor);
* weight compute-copies are re-derived inside the graph (``recompute_weight_copies``) so replays see the
  optimizer's updates;
* dropout draws from a device-resident counter advanced by the kernels (new masks every replay);
* the DDP wrapper runs in ``overlap=False`` mode (bucket all-reduces issued after backward on the
  capturing stream) -- RCCL collectives are capturable.

:class:`CapturedSteps` records SEVERAL consecutive steps into one graph, each reading its own persistent
input batch (e.g. slices of an HBM-resident dataset, so no per-step input copy exists at all).  One replay
then runs all of them: the host-side replay cost (~10 us per graph launch on MI355X) is paid once per
group instead of once per step, which matters for the MNIST nets whose whole step is ~60-80 us.  Every
captured step is a complete training step (forward, backward, all-reduce, optimizer update).
"""
from __future__ import annotations

import torch

from ..ops import functional as OF


def upload(g: torch.cuda.CUDAGraph) -> None:
    """hipGraphUpload the instantiated graph (its launch resources are set up now, so the first replay -- the
    first step of a timed region -- does not pay for them).  Best effort: a runtime without it is left as is."""
    try:
        from .. import _native

        _native.C().graph_upload(int(g.raw_cuda_graph_exec()))
        torch.cuda.synchronize()
    except Exception:  # noqa: BLE001 - an optimisation only
        pass


class CapturedStep:
    def __init__(self, step_fn, example_inputs, warmup: int = 3):
        self.step_fn = step_fn
        # static inputs are leaves: an input that requires grad (a pipeline stage's activation) gets its
        # gradient in .grad of the static buffer, not through a CloneBackward into the caller's tensor
        self.static_inputs = [t.detach().clone().requires_grad_(t.requires_grad) for t in example_inputs]
        self.graph = None
        self.static_out = None
        self._warmup = warmup

    def capture(self):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(self._warmup):
                self.step_fn(*self.static_inputs)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with OF.recompute_weight_copies():
            with torch.cuda.graph(g):
                self.static_out = self.step_fn(*self.static_inputs)
        torch.cuda.synchronize()
        upload(g)
        self.graph = g
        return self

    def __call__(self, *inputs):
        with torch.no_grad():  # (a static input may be a leaf that requires grad)
            for dst, src in zip(self.static_inputs, inputs):
                if dst.data_ptr() != src.data_ptr():
                    dst.copy_(src, non_blocking=True)
        self.graph.replay()
        return self.static_out


class CapturedSteps:
    """``len(batches)`` consecutive training steps in ONE hipGraph; step ``i`` reads ``batches[i]`` in place.

    ``batches`` must stay alive and unchanged in address for the graph's lifetime (dataset slices are).
    ``replay()`` runs the whole group and returns the last step's output."""

    def __init__(self, step_fn, batches, warmup: int = 3, pool=None, prologue=None):
        self.step_fn = step_fn
        self.prologue = prologue  # recorded before the steps (e.g. a device-counter batch gather into the slots)
        self.batches = [tuple(b) for b in batches]
        self.graph = None
        self.outputs = None
        self._warmup = warmup
        self._pool = pool  # a graph memory pool shared with graphs that never replay concurrently with this one

    @property
    def steps(self) -> int:
        return len(self.batches)

    def capture(self):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for i in range(self._warmup):
                self.step_fn(*self.batches[i % len(self.batches)])
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with OF.recompute_weight_copies():
            with torch.cuda.graph(g, pool=self._pool):
                if self.prologue is not None:
                    self.prologue()
                self.outputs = [self.step_fn(*b) for b in self.batches]
        torch.cuda.synchronize()
        upload(g)
        self.graph = g
        return self

    def replay(self):
        self.graph.replay()
        return self.outputs[-1]
