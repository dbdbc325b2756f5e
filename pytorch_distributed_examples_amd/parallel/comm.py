"""The GPU data plane of a data-parallel job, chosen once.

``data_plane(ctx)`` returns the communicator plug-in for :class:`.ddp.DistributedDataParallel`:

* world 1 or CPU / gloo: ``None`` (DDP uses the c10d group, or nothing at world 1);
* GPUs over RCCL: a :class:`.rccl.StreamComm` (stream-ordered, hipGraph-capturable RCCL all-reduce) wrapped in
  a :class:`.xgmi_allreduce.RoutedComm` that sends latency-bound buckets (<= ``PDE_XGMI_THRESHOLD``, 1 MiB)
  through the one-shot xGMI peer all-reduce.  ``PDE_XGMI=0`` keeps every bucket on RCCL.
"""
from __future__ import annotations

import os


def data_plane(ctx, group=None):
    if ctx.device.type != "cuda" or ctx.world_size <= 1 or ctx.backend != "nccl":
        return None
    from .rccl import StreamComm

    comm = StreamComm(ctx.device, group=group)
    if os.environ.get("PDE_XGMI", "1") == "0":
        return comm
    from .xgmi_allreduce import RoutedComm, XgmiAllreduce

    return RoutedComm(comm, XgmiAllreduce(ctx.device, group=group))
