"""Horovod-compatible core API on the MI355X runtime.

``init()`` joins the job (torchrun env, the elastic driver's rendezvous, or a 1-process world).  Like
Horovod (Gloo controller + NCCL data plane), the CONTROL plane is always CPU/gloo and the GPU DATA plane
is RCCL:

* the default process group is gloo (object broadcasts, barriers, elastic host-update checks), so a dead
  peer surfaces as a connection error -- never as a hung or watchdog-aborted GPU collective;
* the C++ tensor-fusion engine (:class:`_comm.FusionEngine`) gets a DEDICATED gloo group for its
  negotiation cycles (and the CPU data plane), used only from the engine thread;
* on GPUs the engine drives an RCCL communicator of our own (:class:`_comm.RcclComm`, unique id exchanged
  through the c10d store) on a high-priority stream.

Collectives return handles; ``synchronize(handle)`` orders the caller's stream after the collective (GPU)
or blocks (CPU); engine failures raise :class:`HorovodInternalError`.  Environment knobs (Horovod names
where one exists):

    HOROVOD_FUSION_THRESHOLD   fusion buffer bytes (default: xGMI policy, 64 MiB cap)
    HOROVOD_CYCLE_TIME         negotiation cycle in ms (default 0.5)
    HOROVOD_TIMELINE           Chrome-trace file written by the engine
    PDE_HVD_TIMEOUT            seconds before a stuck collective / control cycle is declared failed (300)
    PDE_HVD_BLOCKING_WAIT      1: synchronize() polls GPU completion on the host with liveness checks
                               (default on under the elastic driver, so failures raise from synchronize)
    HOROVOD_CACHE_CAPACITY     response-cache entries (0: negotiate every request by name)
    PDE_HVD_DATA_PLANE         auto (RCCL + one-shot xGMI for fused batches <= PDE_XGMI_THRESHOLD bytes) |
                               rccl | xgmi (no RCCL: ranks rehearsing on ONE GPU, where RCCL refuses to run)
"""
from __future__ import annotations

import contextlib
import datetime
import os
import threading

import torch
import torch.distributed as dist

from .. import _native
from ..elastic import rendezvous
from ..parallel import xgmi
from .exceptions import HorovodInternalError


class ReduceOp:
    Sum = 0
    Average = 1
    Min = 2
    Max = 3
    Product = 4
    Adasum = 10


Average, Sum, Adasum, Min, Max, Product = (ReduceOp.Average, ReduceOp.Sum, ReduceOp.Adasum, ReduceOp.Min,
                                            ReduceOp.Max, ReduceOp.Product)

_DIST_OPS = {ReduceOp.Sum: dist.ReduceOp.SUM, ReduceOp.Min: dist.ReduceOp.MIN, ReduceOp.Max: dist.ReduceOp.MAX,
             ReduceOp.Product: dist.ReduceOp.PRODUCT}


class _Ctx:
    def __init__(self):
        self.initialized = False
        self.rank = 0
        self.size = 1
        self.local_rank = 0
        self.local_size = 1
        self.device = torch.device("cpu")
        self.engine = None
        self.comm = None
        self.xgmi = None
        self.group = None
        self.engine_group = None
        self.owns_pg = False
        self.rdzv = None
        self.generation = 0
        self.names: dict = {}
        self.lock = threading.Lock()


_ctx = _Ctx()


def _fusion_bytes(world: int) -> int:
    env = os.environ.get("HOROVOD_FUSION_THRESHOLD")
    if env:
        return int(env)
    # one fusion buffer carries >= the xGMI bucket floor; Horovod's 64 MiB default as the cap
    return max(xgmi.bucket_floor(max(world, 2)), min(xgmi.MAX_BUCKET_BYTES, 64 * 2 ** 20))


# engines whose thread could not be joined after an abort (stuck in a control cycle with a dead peer):
# kept alive so the detached thread never touches freed memory
_retired: list = []


def _py_allreduce(t, op):
    group = _ctx.engine_group
    if op == ReduceOp.Average:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        t.div_(_ctx.size)
    else:
        dist.all_reduce(t, op=_DIST_OPS[op], group=group)


def _py_broadcast(t, root):
    dist.broadcast(t, root, group=_ctx.engine_group)


def _py_allgather(t, out):
    dist.all_gather_into_tensor(out, t, group=_ctx.engine_group)


def init(comm=None, device: str | None = None):
    """Initialise (or re-initialise after an elastic reset) the job."""
    if _ctx.initialized:
        return
    use_gpu = device != "cpu" and torch.cuda.is_available()
    backend = "gloo"  # control plane; the GPU data plane is the engine's own RCCL communicator
    timeout = datetime.timedelta(seconds=int(os.environ.get("PDE_HVD_TIMEOUT", "300")))
    if rendezvous.elastic_env():
        if _ctx.rdzv is None:
            _ctx.rdzv = rendezvous.RendezvousClient()
        rnd, rank, size = _ctx.rdzv.join()
        local_rank = int(os.environ.get("LOCAL_RANK", os.environ.get("PDE_WORKER_ID", "0")))
        if use_gpu:
            torch.cuda.set_device(local_rank % torch.cuda.device_count())
        store = _ctx.rdzv.pg_store()
        dist.init_process_group(backend, store=store, rank=rank, world_size=size, timeout=timeout)
        _ctx.owns_pg = True
        _ctx.generation = rnd
    else:
        from ..parallel import dist as pdist

        _ctx.owns_pg = not dist.is_initialized()
        ctx = pdist.init_distributed(backend=backend, device="cpu" if not use_gpu else None,
                                     timeout_s=int(timeout.total_seconds()))
        rank, size, local_rank = ctx.rank, ctx.world_size, ctx.local_rank
        store = dist.distributed_c10d._get_default_store()
    _ctx.rank, _ctx.size = dist.get_rank(), dist.get_world_size()
    _ctx.local_rank = local_rank
    _ctx.local_size = int(os.environ.get("LOCAL_WORLD_SIZE", str(_ctx.size)))
    _ctx.device = torch.device("cuda", torch.cuda.current_device()) if use_gpu else torch.device("cpu")
    # control plane: the default group when it is gloo, else (an application that initialised RCCL/NCCL
    # itself) a gloo group over the same ranks
    _ctx.group = dist.group.WORLD if dist.get_backend() == "gloo" else dist.new_group(backend="gloo", timeout=timeout)
    # the engine thread's own group: its negotiation collectives never interleave with the main thread's
    _ctx.engine_group = dist.new_group(backend="gloo", timeout=timeout) if _ctx.size > 1 else _ctx.group
    C = _native.comm()
    tl = os.environ.get("HOROVOD_TIMELINE", "")
    if tl and _ctx.size > 1:
        tl = f"{tl}.rank{_ctx.rank}"
    cycle_ms = float(os.environ.get("HOROVOD_CYCLE_TIME", "0.5"))
    eng = C.FusionEngine(_ctx.rank, _ctx.size, _fusion_bytes(_ctx.size), tl, cycle_ms)
    eng.set_py_backend(_py_allreduce, _py_broadcast, _py_allgather)
    if _ctx.size > 1:
        eng.set_control(_ctx.engine_group)
    eng.set_timeout(float(timeout.total_seconds()))
    blocking = os.environ.get("PDE_HVD_BLOCKING_WAIT")
    eng.set_blocking_wait(blocking == "1" if blocking is not None else rendezvous.elastic_env())
    if use_gpu:
        plane = os.environ.get("PDE_HVD_DATA_PLANE", "auto")
        # several ranks on one device (a one-GPU rehearsal): RCCL refuses duplicate devices -> xGMI only
        shared = _ctx.size > 1 and torch.cuda.device_count() < _ctx.local_size
        if plane == "rccl" or (plane == "auto" and not shared):
            key = f"pde/hvd/rccl_uid/{_ctx.generation}"
            if _ctx.rank == 0:
                store.set(key, C.rccl_unique_id())
            uid = store.get(key)
            comm = C.RcclComm()
            comm.init(uid, _ctx.rank, _ctx.size, _ctx.device.index, True)
            eng.set_rccl(comm)
            _ctx.comm = comm
        # the one-shot exchange maps every peer's buffer over IPC: one node only (a multi-host job stays on
        # RCCL, whose transport spans hosts)
        single_node = _ctx.local_size == _ctx.size
        if _ctx.size > 1 and (plane == "xgmi" or (plane == "auto" and single_node)):
            # latency-bound fused batches (the CNN's 87 KB of gradients) take the one-shot peer exchange
            from ..parallel.xgmi_allreduce import DEFAULT_THRESHOLD, XgmiAllreduce

            _ctx.xgmi = XgmiAllreduce(_ctx.device, key=f"hvd/{_ctx.generation}")
            eng.set_xgmi(_ctx.xgmi.impl, DEFAULT_THRESHOLD if plane == "auto" else _ctx.xgmi.max_bytes)
    _ctx.engine = eng
    _ctx.names = {}
    _ctx.watch = None
    if rendezvous.elastic_env() and _ctx.xgmi is not None:
        # the driver reports a dead member of this round at once: spinning xGMI exchanges give up on the host
        # abort word (elastic/rewire.py _FailureWatch) and the engine raises HorovodInternalError at the next
        # synchronize / commit -- detection in ~0.1 s instead of the exchange timeout
        from ..elastic.rewire import _FailureWatch

        _ctx.watch = _FailureWatch(_ctx.rdzv, _ctx.generation, _ctx.xgmi)
    _ctx.initialized = True


def shutdown(abort: bool = False):
    """Tear down the engine, communicator and process group (in-process; used by elastic reset)."""
    if not _ctx.initialized:
        return
    if getattr(_ctx, "watch", None) is not None:
        _ctx.watch.stop()
        _ctx.watch = None
    try:
        _ctx.engine.shutdown(abort)
    except Exception:  # noqa: BLE001 - a failed peer may leave the engine in an error state
        pass
    if abort:
        _retired.append(_ctx.engine)
    if _ctx.comm is not None:
        if abort:
            _ctx.comm.abort()
        else:
            try:
                _ctx.comm.destroy()
            except Exception:  # noqa: BLE001
                _ctx.comm.abort()
    if _ctx.xgmi is not None:
        try:
            _ctx.xgmi.close()
        except Exception:  # noqa: BLE001 - a dead peer's mapping may refuse a clean close
            pass
    _ctx.engine = None
    _ctx.comm = None
    _ctx.xgmi = None
    _ctx.engine_group = None
    try:
        if dist.is_initialized() and _ctx.owns_pg:
            dist.destroy_process_group()
    except Exception:  # noqa: BLE001
        pass
    _ctx.owns_pg = False
    _ctx.initialized = False


def is_initialized() -> bool:
    return _ctx.initialized


def _need():
    if not _ctx.initialized:
        raise ValueError("Horovod has not been initialized; use hvd.init().")


def size() -> int:
    _need()
    return _ctx.size


def rank() -> int:
    _need()
    return _ctx.rank


def local_rank() -> int:
    _need()
    return _ctx.local_rank


def local_size() -> int:
    _need()
    return _ctx.local_size


def cross_rank() -> int:
    return rank() // max(1, local_size())


def cross_size() -> int:
    return max(1, size() // max(1, local_size()))


def is_homogeneous() -> bool:
    return True


def rocm_built() -> bool:
    return torch.version.hip is not None


def nccl_built() -> bool:  # RCCL == NCCL API on ROCm
    return True


def mpi_built() -> bool:
    return False


def gloo_built() -> bool:
    return True


def gpu_available(framework: str = "torch") -> bool:
    return torch.cuda.is_available()


# ---------------------------------------------------------------------------------------------
# handles / collectives
# ---------------------------------------------------------------------------------------------
class _Handle:
    __slots__ = ("h", "output", "post")

    def __init__(self, h, output, post=None):
        self.h, self.output, self.post = h, output, post


def _enqueue(fn, *args):
    """Engine enqueue; a failed engine (dead peer, aborted communicator) raises HorovodInternalError."""
    try:
        return fn(*args)
    except RuntimeError as exc:
        msg = str(exc)
        if msg.startswith("HorovodInternalError") or "has been shut down" in msg:
            raise HorovodInternalError(msg.split("\n")[0]) from exc
        raise


def _auto_name(prefix: str, name: str | None) -> str:
    if name is not None:
        return name
    with _ctx.lock:
        n = _ctx.names.get(prefix, 0)
        _ctx.names[prefix] = n + 1
    return f"{prefix}.noname.{n}"


def _resolve_op(average, op):
    if op is None:
        op = ReduceOp.Average if (average is None or average) else ReduceOp.Sum
    if op == ReduceOp.Adasum:
        raise NotImplementedError("Adasum is not supported; use Average or Sum")
    return op


def allreduce_async_(tensor, average=None, name=None, op=None, prescale_factor=1.0, postscale_factor=1.0,
                     compression_bf16: bool = False):
    _need()
    op = _resolve_op(average, op)
    t = tensor if tensor.is_contiguous() else tensor.contiguous()
    h = _enqueue(_ctx.engine.allreduce, t, t, _auto_name("allreduce", name), op, float(prescale_factor),
                 float(postscale_factor), compression_bf16)
    post = None if t is tensor else (lambda out, tensor=tensor: tensor.copy_(out))
    return _Handle(h, t, post)


def allreduce_async(tensor, average=None, name=None, op=None, prescale_factor=1.0, postscale_factor=1.0):
    _need()
    op = _resolve_op(average, op)
    t = tensor.contiguous()
    out = torch.empty_like(t)
    h = _enqueue(_ctx.engine.allreduce, t, out, _auto_name("allreduce", name), op, float(prescale_factor),
                 float(postscale_factor), False)
    return _Handle(h, out)


def allreduce(tensor, average=None, name=None, compression=None, op=None, prescale_factor=1.0,
              postscale_factor=1.0):
    if compression is not None:
        c, ctx = compression.compress(tensor)
        out = synchronize(allreduce_async(c, average, name, op, prescale_factor, postscale_factor))
        return compression.decompress(out, ctx)
    return synchronize(allreduce_async(tensor, average, name, op, prescale_factor, postscale_factor))


def allreduce_(tensor, average=None, name=None, op=None, prescale_factor=1.0, postscale_factor=1.0):
    return synchronize(allreduce_async_(tensor, average, name, op, prescale_factor, postscale_factor))


def grouped_allreduce(tensors, average=None, name=None, op=None):
    hs = [allreduce_async(t, average, f"{name}.{i}" if name else None, op) for i, t in enumerate(tensors)]
    return [synchronize(h) for h in hs]


def allgather_async(tensor, name=None):
    _need()
    h = _enqueue(_ctx.engine.allgather, tensor.contiguous(), _auto_name("allgather", name))
    return _Handle(h, None)


def allgather(tensor, name=None):
    return synchronize(allgather_async(tensor, name))


def broadcast_async_(tensor, root_rank, name=None):
    _need()
    t = tensor if tensor.is_contiguous() else tensor.contiguous()
    h = _enqueue(_ctx.engine.broadcast, t, int(root_rank), _auto_name("broadcast", name))
    post = None if t is tensor else (lambda out, tensor=tensor: tensor.copy_(out))
    return _Handle(h, t, post)


def broadcast_async(tensor, root_rank, name=None):
    return broadcast_async_(tensor.clone(), root_rank, name)


def broadcast_(tensor, root_rank, name=None):
    return synchronize(broadcast_async_(tensor, root_rank, name))


def broadcast(tensor, root_rank, name=None):
    return synchronize(broadcast_async(tensor, root_rank, name))


def alltoall(tensor, splits=None, name=None):
    """All-to-all along dim 0.  GPU: RCCL (``ncclAllToAll`` for equal splits, grouped send/recv
    otherwise); CPU: gloo.  Split sizes are exchanged over the gloo control plane."""
    _need()
    t = tensor.contiguous()
    rows = t.shape[0] if t.dim() else 1
    if splits is None:
        if rows % _ctx.size:
            raise ValueError("alltoall without splits needs dim 0 divisible by the world size")
        splits = [rows // _ctx.size] * _ctx.size
    splits = [int(s) for s in splits]
    if sum(splits) != rows:
        raise ValueError("alltoall splits must sum to dim 0")
    all_splits = allgather_object(splits)
    out_splits = [int(s[_ctx.rank]) for s in all_splits]
    out = t.new_empty((sum(out_splits),) + tuple(t.shape[1:]))
    if t.is_cuda:
        row = max(1, t[0].numel()) if rows else 1
        comm = _ctx.comm
        if len(set(splits)) == 1 and len(set(out_splits)) == 1:
            res = comm.alltoall(t.reshape(-1))
            return res.view_as(out)
        comm.group_start()
        soff = roff = 0
        for peer in range(_ctx.size):
            if splits[peer]:
                comm.send(t.reshape(-1)[soff * row:(soff + splits[peer]) * row], peer)
            if out_splits[peer]:
                comm.recv(out.reshape(-1)[roff * row:(roff + out_splits[peer]) * row], peer)
            soff += splits[peer]
            roff += out_splits[peer]
        comm.group_end()
        return out
    dist.all_to_all_single(out, t, out_splits, splits, group=_ctx.group)
    return out


def synchronize(handle):
    _need()
    if not isinstance(handle, _Handle):
        raise ValueError("synchronize expects a handle returned by an *_async op")
    try:
        out = _ctx.engine.wait(handle.h)
    except RuntimeError as exc:
        raise HorovodInternalError(str(exc).split("\n")[0]) from exc
    if handle.post is not None:
        handle.post(out)
        return handle.output if handle.output is not None else out
    return out


def poll(handle) -> bool:
    _need()
    return bool(_ctx.engine.poll(handle.h))


def join(device=-1) -> int:
    """Barrier; returns the last rank to join (Horovod semantics for uneven inputs, simplified)."""
    _need()
    t = torch.tensor([_ctx.rank], dtype=torch.float32)
    with _control_plane("join"):
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=_ctx.group)
    return int(t.item())


def barrier():
    _need()
    if _ctx.size > 1:
        with _control_plane("barrier"):
            dist.barrier(group=_ctx.group)


def broadcast_object(obj, root_rank=0, name=None):
    _need()
    if _ctx.size == 1:
        return obj
    lst = [obj if _ctx.rank == root_rank else None]
    with _control_plane("broadcast_object"):
        dist.broadcast_object_list(lst, src=root_rank, group=_ctx.group)
    return lst[0]


def allgather_object(obj, name=None):
    _need()
    out = [None] * _ctx.size
    with _control_plane("allgather_object"):
        dist.all_gather_object(out, obj, group=_ctx.group)
    return out


@contextlib.contextmanager
def _control_plane(what: str):
    """Failures of the gloo control plane are peer failures by construction (a dead or unreachable rank:
    connection reset, closed pair, store timeout): typed as HorovodInternalError HERE, at the source, so
    ``hvd.elastic.run`` never has to guess from message text."""
    try:
        yield
    except HorovodInternalError:
        raise
    except (RuntimeError, ConnectionError, TimeoutError) as exc:  # c10d DistError subclasses RuntimeError
        raise HorovodInternalError(f"control plane ({what}): {str(exc).splitlines()[0] if str(exc) else exc!r}") \
            from exc


def check_health():
    """Raise HorovodInternalError if the GPU data plane reported a failure that no engine cycle saw: a
    timed-out xGMI exchange inside a replayed graph (graph mode bypasses the engine thread).  A plain read
    of host-mapped status words: call it at every commit / step boundary."""
    _need()
    _enqueue(_ctx.engine.check_xgmi)


def set_graph_mode(on: bool, tensors=()):
    """Engine side of :meth:`DistributedOptimizer.enable_graph_mode`: size the inline staging buffer once
    for ``tensors`` and park the idle negotiation loop (no lockstep bit all-reduces while replays run)."""
    _need()
    _ctx.engine.set_graph_mode(bool(on), list(tensors))


def allreduce_inline_(tensors, op=ReduceOp.Average, prescale_factor=1.0, postscale_factor=1.0,
                      compression_bf16=False):
    """Graph mode: all-reduce ``tensors`` in place on the CURRENT stream, batched exactly as the engine would,
    without the negotiation cycle (stream-ordered, no host wait, hipGraph-capturable).  Every rank must make the
    same call with the same tensors in the same order -- what a cached (already negotiated) tensor set
    guarantees; :meth:`DistributedOptimizer.enable_graph_mode` checks that first."""
    _need()
    _enqueue(_ctx.engine.allreduce_inline, list(tensors), int(op), float(prescale_factor), float(postscale_factor),
             bool(compression_bf16))


def is_cached(name: str) -> bool:
    """Whether ``name`` is in the engine's response cache (negotiated with the same signature before)."""
    _need()
    return bool(_ctx.engine.cached(name))


def engine_stats() -> dict:
    _need()
    return dict(_ctx.engine.stats())
