"""Data-parallel wrapper with xGMI-sized gradient buckets (SURVEY.md P1, §2.6 DDP rows, §5.8).

Mirrors ``torch.nn.parallel.DistributedDataParallel`` as used by the reference
(pytorch_elastic/mnist_ddp_elastic.py:58, rpc/server_model_data_parallel.py:41):

* construction broadcasts parameters and buffers from rank 0 -- coalesced into ONE flat broadcast;
* gradients live in one flat fp32 buffer laid out in bucket order (``param.grad`` are views into it), so
  a bucket is a single contiguous tensor and ``zero_grad`` is a single fill;
* a post-accumulate-grad hook counts down each bucket; full buckets are all-reduced asynchronously, in
  bucket order (the same on every rank), while the rest of backward runs -- RCCL runs them on its own
  stream, ordered after the producing kernels;
* RCCL averages in-collective (``ReduceOp.AVG``), so no separate divide kernel runs (gloo: SUM then a
  scale);
* bucket sizes follow :mod:`.xgmi` (sized for 7 point-to-point links, not DDP's 25 MiB default);
* ``overlap=False`` skips the hooks and reduces every bucket in :meth:`sync_gradients` -- the form used
  inside a captured hipGraph step;
* ``grad_dtype=torch.bfloat16`` halves the bytes on the wire: on the xGMI data plane the casts are fused
  into the one-shot all-reduce kernel and DDP copies nothing; on RCCL each bucket is cast by our HIP kernel
  into a persistent bf16 buffer, all-reduced in place (bf16, AVG in-collective) and cast back by our kernel
  into the flat fp32 gradient -- no allocation and no ATen kernel per bucket;
* ``static_graph=True`` (every step writes every gradient through the same kernels): once two consecutive steps
  saw each gradient view's first writer STORE (``ops.functional._sink_accum`` consumed the view's zero-filled
  mark), ``zero_grad`` stops filling the flat gradient -- the first writers overwrite it anyway.  The mark is still
  set every step and checked BEFORE the gradients are used: when a bucket is reduced (and in ``sync_gradients`` at
  world 1) a view whose mark survived a skipped-fill step got no gradient this step, so it is zeroed there (an
  unused parameter's gradient is zero, as in a filled step) and the next ``zero_grad`` fills again.  A
  ``zero_grad`` with no backward since the last one consumed no mark: it fills (the buffer may hold an old step);
* ``comm=`` swaps the c10d group for another communicator (``size``, ``supports_avg``,
  ``allreduce_async(t, avg) -> work``, ``broadcast_(t, src)``), e.g. the per-round RCCL communicator of
  :mod:`..elastic.rewire` that is aborted and rebuilt in-process on a membership change.
"""
from __future__ import annotations

import contextlib

import torch
import torch.distributed as dist
from torch import nn

from ..ops import streams
from . import xgmi


def _flat_broadcast(tensors, src, group, comm=None):
    if not tensors:
        return
    by_dtype: dict = {}
    for t in tensors:
        by_dtype.setdefault((t.dtype, t.device), []).append(t)
    for (dtype, device), ts in by_dtype.items():
        flat = torch.cat([t.detach().reshape(-1) for t in ts])
        if comm is not None:
            comm.broadcast_(flat, src)
        else:
            dist.broadcast(flat, src, group=group)
        off = 0
        with torch.no_grad():
            for t in ts:
                n = t.numel()
                t.copy_(flat[off:off + n].view_as(t))
                off += n


def _cast(src: torch.Tensor, dst: torch.Tensor) -> None:
    """fp32 <-> bf16 bucket cast: our HIP kernels on GPU (pytorch_distributed_examples_amd._C), ATen on CPU."""
    if src.is_cuda:
        from .. import _native

        C = _native.C()
        (C.cast_bf16_into if src.dtype == torch.float32 else C.cast_f32_into)(src, dst)
    else:
        dst.copy_(src)


class DistributedDataParallel(nn.Module):
    def __init__(self, module: nn.Module, process_group=None, bucket_cap_mb: float | None = None,
                 broadcast_buffers: bool = True, overlap: bool = True, grad_dtype: torch.dtype | None = None,
                 src_rank: int = 0, param_order: str = "reverse", comm=None, static_graph: bool = False):
        super().__init__()
        self.module = module
        self.pg = process_group
        self.comm = comm
        if comm is not None:
            self.world = comm.size
        else:
            self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.broadcast_buffers = broadcast_buffers
        self.overlap = overlap
        self.grad_dtype = grad_dtype
        # src_rank is a rank WITHIN the group; c10d broadcast wants the global rank
        self.src = dist.get_global_rank(process_group, src_rank) if (process_group is not None and comm is None and
                                                                     dist.is_initialized()) else src_rank
        self._params = [p for p in module.parameters() if p.requires_grad]
        dev = self._params[0].device if self._params else torch.device("cpu")
        if comm is not None:
            self._use_avg = bool(comm.supports_avg)
        else:
            self._use_avg = dist.is_initialized() and dist.get_backend(process_group) == "nccl"
        if self.world > 1:
            _flat_broadcast(list(module.parameters()) + list(module.buffers()), self.src, process_group, comm)

        # bucket plan over parameters in reverse registration order (~ gradient ready order).
        # param_order="forward" lays the flat gradient out in registration order instead, so a fused
        # whole-model kernel that produces all gradients at once can write it directly.
        order = list(reversed(self._params)) if param_order == "reverse" else list(self._params)
        # Every gradient view starts on a 256-byte boundary (64 fp32), so the kernels that read or write it (the
        # fused optimiser, GEMM epilogues) take their 16-byte vector paths: one odd-sized tensor early in the
        # layout (a 10-wide bias) would otherwise misalign every view after it -- the MLP's Adam ran its scalar
        # path on all 5M parameters (r4n: 52 us).  The "forward" layout stays dense: it IS the fused CNN kernel's
        # flat parameter order.  Padding elements are never written (zero) and ride along in the all-reduce.
        align = 64 if param_order == "reverse" else 1
        padded = [-(-p.numel() // align) * align for p in order]
        sizes = [n * (2 if grad_dtype == torch.bfloat16 else 4) for n in padded]
        cap = int(bucket_cap_mb * 2 ** 20) if bucket_cap_mb else None
        plan = xgmi.plan_buckets(sizes, self.world, cap)
        total = sum(padded)
        self.flat_grad = torch.zeros(total, dtype=torch.float32, device=dev)
        self._views = {}
        self._bucket_of = {}
        self._bucket_ranges = []
        off = 0
        for bi, idxs in enumerate(plan):
            start = off
            for i in idxs:
                p = order[i]
                n = p.numel()
                self._views[p] = self.flat_grad[off:off + n].view_as(p)
                self._bucket_of[p] = bi
                off += padded[i]
            self._bucket_ranges.append((start, off))
        self._bucket_sizes = [len(idxs) for idxs in plan]
        self._bucket_params = [[order[i] for i in idxs] for idxs in plan]
        for p in self._params:
            p.grad = self._views[p]
        self._bucket_flat = [self.flat_grad[s:e] for s, e in self._bucket_ranges]
        self._bf16_bufs = [torch.empty(e - s, dtype=torch.bfloat16, device=dev) for s, e in self._bucket_ranges] \
            if grad_dtype == torch.bfloat16 else None
        self._sync = True
        self.static_graph = static_graph
        self._covered = 0       # consecutive steps whose every gradient view was stored by its first writer
        self._filled = True     # the last zero_grad filled
        self._marked = False    # the views carry zero_grad's marks
        self.fills_skipped = 0
        self.stale_zeroed = 0   # views zeroed at reduction time: unwritten in a skipped-fill step
        self._reset_state()
        self._hooks = []
        if overlap and self.world > 1:
            for p in self._params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(p)))

    # ------------------------------------------------------------------------------------------
    def _reset_state(self):
        self._pending = list(self._bucket_sizes)
        self._next = 0
        self._works = []
        self._callback_queued = False

    def _make_hook(self, p):
        view = self._views[p]

        def hook(param):
            if not self._sync:
                return
            if param.grad is None or param.grad.data_ptr() != view.data_ptr():
                # someone replaced .grad (e.g. zero_grad(set_to_none=True)): fold it back into the bucket
                if param.grad is not None:
                    view.copy_(param.grad)
                param.grad = view
            if not self._callback_queued:
                self._callback_queued = True
                torch.autograd.Variable._execution_engine.queue_callback(self._finalize_overlap)
            b = self._bucket_of[param]
            self._pending[b] -= 1
            self._launch_ready()

        return hook

    def _repair_stale(self, b: int):
        """Before bucket ``b``'s gradients are used: in a step whose zero fill was skipped, zero every view that no
        storing first writer consumed (it still holds an older step's gradient)."""
        if not self.static_graph or self._filled or not self._marked:
            return
        for p in self._bucket_params[b]:
            v = self._views[p]
            if v.__dict__.pop("_pde_fresh", False):
                v.zero_()
                self.stale_zeroed += 1
                self._covered = -1  # the next zero_grad fills (and the coverage count restarts)

    def _launch(self, b: int):
        self._repair_stale(b)
        if self.flat_grad.is_cuda:  # weight gradients may still be running on the side stream (ops/streams.py)
            streams.join(self.flat_grad.device)
        fused_wire = getattr(self.comm, "fuses_bf16_wire", None)
        if self._bf16_bufs is not None and fused_wire is not None and fused_wire(self._bucket_flat[b]):
            # the communicator casts on the wire itself (fused into the xGMI one-shot kernel): no copies here
            work = self.comm.allreduce_async(self._bucket_flat[b], avg=self._use_avg, wire_bf16=True)
            self._works.append((-1 - b, work))
            return
        if self._bf16_bufs is not None:
            buf = self._bf16_bufs[b]
            _cast(self._bucket_flat[b], buf)
        else:
            buf = self._bucket_flat[b]
        if self.comm is not None:
            work = self.comm.allreduce_async(buf, avg=self._use_avg)
        else:
            op = dist.ReduceOp.AVG if self._use_avg else dist.ReduceOp.SUM
            work = dist.all_reduce(buf, op=op, group=self.pg, async_op=True)
        self._works.append((b, work))

    def _launch_ready(self):
        while self._next < len(self._pending) and self._pending[self._next] <= 0:
            self._launch(self._next)
            self._next += 1

    def _complete(self):
        for b, work in self._works:
            work.wait()
            if self._bf16_bufs is not None and b >= 0:  # b < 0: reduced in place with a bf16 wire
                _cast(self._bf16_bufs[b], self._bucket_flat[b])
        if not self._use_avg and self.world > 1:
            self.flat_grad.mul_(1.0 / self.world)
        self._reset_state()

    def _finalize_overlap(self):
        # buckets whose params got no gradient this step (unused parameters) still reduce
        while self._next < len(self._pending):
            self._launch(self._next)
            self._next += 1
        self._complete()

    # ------------------------------------------------------------------------------------------
    def sync_gradients(self):
        """Reduce all buckets now (non-overlapped mode / after ``no_sync`` accumulation)."""
        if self.world <= 1:
            for b in range(len(self._bucket_ranges)):
                self._repair_stale(b)
            return
        for b in range(len(self._bucket_ranges)):
            self._launch(b)
        self._complete()

    def forward(self, *args, **kwargs):
        if self.broadcast_buffers and self.world > 1 and self.module.training:
            bufs = [b for b in self.module.buffers() if b.is_floating_point()]
            if bufs:
                _flat_broadcast(bufs, self.src, self.pg, self.comm)
        return self.module(*args, **kwargs)

    def zero_grad(self, set_to_none: bool = False):
        skip = False
        if self.static_graph and self._marked:
            left = [p for p in self._params if self._views[p].__dict__.get("_pde_fresh", False)]
            if len(left) == len(self._params):
                pass  # no backward since the last zero_grad: nothing consumed, fill (below) without counting a step
            elif self._covered < 0:
                self._covered = 0  # stale views were zeroed at reduction time in the last step
            else:
                self._covered = 0 if left else self._covered + 1
            skip = self._covered >= 2 and len(left) < len(self._params)
        if skip:
            self.fills_skipped += 1
        else:
            self.flat_grad.zero_()
        self._filled = not skip
        for p in self._params:
            if p.grad is None or p.grad.data_ptr() != self._views[p].data_ptr():
                p.grad = self._views[p]
            # zero-filled: the first weight-gradient kernel of the step may store instead of add
            # (ops.functional._sink_accum; bitwise the same as adding to zero, no read-modify-write)
            p.grad.__dict__["_pde_fresh"] = True
        self._marked = True

    def remove_hooks(self):
        """Detach from the parameters (before wrapping the same module in a new DDP, e.g. per round)."""
        for h in self._hooks:
            h.remove()
        self._hooks = []

    @contextlib.contextmanager
    def no_sync(self):
        old = self._sync
        self._sync = False
        try:
            yield
        finally:
            self._sync = old

    @property
    def bucket_bytes(self):
        mult = 2 if self.grad_dtype == torch.bfloat16 else 4
        return [(e - s) * mult for s, e in self._bucket_ranges]

    def state_dict(self, *a, **k):
        return self.module.state_dict(*a, **k)

    def load_state_dict(self, *a, **k):
        return self.module.load_state_dict(*a, **k)
