"""The GPU data plane of a data-parallel job, chosen once.

``data_plane(ctx)`` returns the communicator plug-in for :class:`.ddp.DistributedDataParallel`:

* world 1 or CPU / gloo: ``None`` (DDP uses the c10d group, or nothing at world 1);
* GPUs over RCCL: a :class:`.rccl.StreamComm` (stream-ordered, hipGraph-capturable RCCL all-reduce) wrapped in
  a :class:`.xgmi_allreduce.RoutedComm` that sends latency-bound buckets (<= ``PDE_XGMI_THRESHOLD``, 1 MiB)
  through the one-shot xGMI peer all-reduce and, on a single node, larger ones (<= ``PDE_XGMI_TWOSHOT_MB``, 64 MiB)
  through the two-shot xGMI all-reduce (every link carries 2/N of the bucket; RCCL remains the fallback for anything
  larger).  ``PDE_XGMI=0`` keeps every bucket on RCCL; ``PDE_XGMI_TWOSHOT=0`` keeps the large ones there (A/B).
"""
from __future__ import annotations

import os


def data_plane(ctx, group=None, two_shot: bool = True):
    """``two_shot=False``: no two-shot instance (a workload whose gradients all fit the one-shot's 1 MiB buckets --
    the MNIST nets -- would only allocate and hand-shake it)."""
    if ctx.device.type != "cuda" or ctx.world_size <= 1 or ctx.backend != "nccl":
        return None
    from .rccl import StreamComm

    comm = StreamComm(ctx.device, group=group)
    if os.environ.get("PDE_XGMI", "1") == "0":
        return comm
    from .xgmi_allreduce import RoutedComm, XgmiAllreduce

    xgmi2 = None
    single_node = int(os.environ.get("LOCAL_WORLD_SIZE", str(ctx.world_size))) == ctx.world_size
    if two_shot and single_node and os.environ.get("PDE_XGMI_TWOSHOT", "1") != "0":
        mb = float(os.environ.get("PDE_XGMI_TWOSHOT_MB", "64"))
        # (a longer peer-wait bound than the one-shot's 5 s: large buckets are first reduced after the first
        # backward, when ranks may still be far apart from their first-use initialisation)
        xgmi2 = XgmiAllreduce(ctx.device, group=group, max_bytes=int(mb * (1 << 20)), two_shot=True,
                              timeout_s=float(os.environ.get("PDE_XGMI_TIMEOUT_S", "30")))
    return RoutedComm(comm, XgmiAllreduce(ctx.device, group=group), xgmi2=xgmi2)
