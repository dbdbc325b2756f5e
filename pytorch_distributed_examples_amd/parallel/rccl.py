"""Stream-ordered RCCL communicator for the DDP data plane (capturable into hipGraphs).

c10d's ``ProcessGroupNCCL`` cannot be used inside a hipGraph on this ROCm build: its watchdog thread
queries the work's completion event while the capturing stream is live and the process aborts with
``hipErrorStreamCaptureUnsupported`` (measured on MI355X, ``tests/test_comm_gpu.py``).  The gradient
all-reduce of a captured training step therefore goes through our own RCCL communicator
(``csrc/comm/comm_manager.cpp``): ``ncclAllReduce`` enqueued on the caller's CURRENT stream, ordered
after the kernels that produced the gradients and before the optimizer kernel -- no host
synchronisation, no watchdog, nothing that breaks stream capture.  c10d (any backend) stays the control
plane: it exchanges the RCCL unique id through the default store.

Implements the communicator plug-in of :class:`.ddp.DistributedDataParallel` (``comm=``): ``size``,
``rank``, ``supports_avg``, ``allreduce_async(t, avg) -> work`` and ``broadcast_(t, src)``.
"""
from __future__ import annotations

import itertools
import os

import torch
import torch.distributed as dist

from .. import _native

_SEQ = itertools.count()
_RED_SUM, _RED_AVG = 0, 1


class _StreamWork:
    """The collective is stream-ordered: waiting is a no-op for stream consumers."""

    def wait(self):
        return True

    def is_completed(self):
        return True


class _SideWork:
    """An all-reduce enqueued on the communicator's side stream: ``wait()`` makes the CURRENT stream wait
    for it (an event join -- capturable: a fork/join in the hipGraph), never the host."""

    def __init__(self, event, keep):
        self.event, self.keep = event, keep

    def wait(self):
        torch.cuda.current_stream().wait_event(self.event)
        self.keep = None
        return True

    def is_completed(self):
        return self.event.query()


class StreamComm:
    """``side_stream=True``: each all-reduce runs on a dedicated stream forked from the current one, so it
    overlaps whatever the current stream does next (the remaining backward of a pipeline stage); DDP joins
    it in ``_complete`` (work.wait())."""

    def __init__(self, device: torch.device, group=None, side_stream: bool = False):
        assert device.type == "cuda", "StreamComm is the GPU data plane"
        self.rank = dist.get_rank(group)
        self.size = dist.get_world_size(group)
        self.device = device
        self.supports_avg = True
        C = _native.comm()
        # unique id through the default store; the key is unique per communicator and per group
        store = dist.distributed_c10d._get_default_store()
        seq = next(_SEQ)
        ranks = dist.get_process_group_ranks(group) if group is not None else list(range(self.size))
        key = f"pde_stream_comm/{seq}/{'-'.join(map(str, ranks))}"
        if self.rank == 0:
            store.set(key, C.rccl_unique_id())
        uid = store.get(key)
        self.rccl = C.RcclComm()
        self.rccl.init(uid, self.rank, self.size, device.index, True)
        # high priority: a separate hardware queue class, so the spinning all-reduce never shares (and serializes)
        # a queue with the compute stream whose later kernels its peers may be waiting for
        self.side = torch.cuda.Stream(device=device, priority=-1) if side_stream else None
        self._bn_headroom = None
        if self.side is not None:
            # an overlapped all-reduce spins on its side stream while compute (a one-launch BatchNorm) runs:
            # reserve RCCL's workgroups (PDE_RCCL_SIDE_BLOCKS, default 32 channels) out of that kernel's budget
            from ..ops.functional import BnHeadroom

            self._bn_headroom = BnHeadroom(int(os.environ.get("PDE_RCCL_SIDE_BLOCKS", "32")))

    def allreduce_async(self, t: torch.Tensor, avg: bool = False):
        if self.side is None:
            self.rccl.allreduce_(t, _RED_AVG if avg else _RED_SUM)
            return _StreamWork()
        self.side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.side):
            self.rccl.allreduce_(t, _RED_AVG if avg else _RED_SUM)
            ev = torch.cuda.Event()
            ev.record()
        return _SideWork(ev, t)

    def allreduce_(self, t: torch.Tensor, avg: bool = False) -> torch.Tensor:
        self.rccl.allreduce_(t, _RED_AVG if avg else _RED_SUM)
        return t

    def broadcast_(self, t: torch.Tensor, src: int) -> torch.Tensor:
        self.rccl.broadcast_(t, src)
        return t

    def destroy(self):
        if self.rccl is not None:
            self.rccl.destroy()
            self.rccl = None
        if self._bn_headroom is not None:
            self._bn_headroom.release()
            self._bn_headroom = None
