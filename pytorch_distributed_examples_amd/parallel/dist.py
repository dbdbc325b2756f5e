"""Process-group bootstrap (one process per GPU).

Replaces the reference's three bootstraps: torchrun env:// (mnist_ddp_elastic.py:22-27),
``MASTER_ADDR/PORT`` + ``mp.spawn`` (model_parallel_ResNet50.py:229-230) and explicit ``tcp://``
init methods (server_model_data_parallel.py:121-122,155-157).

* backend ``"nccl"`` is RCCL over xGMI on ROCm; ``"gloo"`` is the CPU backend (BASELINE config 0).
  ``backend=None`` picks RCCL when a GPU is present, gloo otherwise.
* ``OMP_NUM_THREADS`` is set BEFORE torch spins up its pool when this module is imported by an entry
  script (quirk Q3: the reference sets it after ``import torch``, which has no effect).
* Rendezvous addresses default to 127.0.0.1 (the container hostname may not resolve).
"""
from __future__ import annotations

import datetime
import os
import socket
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistContext:
    rank: int
    world_size: int
    local_rank: int
    device: torch.device
    backend: str

    @property
    def is_main(self) -> bool:
        return self.rank == 0


_HANDED_OUT: set = set()


def free_port() -> int:
    """A free port not handed out before by this process (two quick calls can otherwise return the same one)."""
    for _ in range(64):
        with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        if port not in _HANDED_OUT:
            _HANDED_OUT.add(port)
            return port
    return port


def free_ports(n: int) -> list:
    """``n`` DISTINCT free ports: every socket stays bound until all are chosen (two back-to-back
    ``free_port()`` calls may hand out the same port, and the second server then fails with EADDRINUSE)."""
    socks = []
    try:
        for _ in range(n):
            s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            s.bind(("127.0.0.1", 0))
            socks.append(s)
        return [s.getsockname()[1] for s in socks]
    finally:
        for s in socks:
            s.close()


def env_int(name: str, default: int) -> int:
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


def init_distributed(backend: str | None = None, device: str | None = None, timeout_s: int = 300,
                     init_method: str | None = None, rank: int | None = None,
                     world_size: int | None = None) -> DistContext:
    """Initialise the default process group from torchrun's env (or as a 1-rank group when launched
    without torchrun) and pin this process to its GPU."""
    rank = env_int("RANK", 0) if rank is None else rank
    world_size = env_int("WORLD_SIZE", 1) if world_size is None else world_size
    local_rank = env_int("LOCAL_RANK", rank)
    use_gpu = (device != "cpu") and torch.cuda.is_available()
    if backend is None:
        # PDE_BACKEND=gloo rehearses a multi-rank GPU job on ONE GPU (ranks share the card; gloo moves
        # the CUDA tensors through the host) -- RCCL refuses two ranks on one device
        backend = os.environ.get("PDE_BACKEND") or ("nccl" if use_gpu else "gloo")
    if use_gpu:
        ndev = torch.cuda.device_count()
        dev = torch.device("cuda", local_rank % max(1, ndev))
        torch.cuda.set_device(dev)
        if env_int("LOCAL_WORLD_SIZE", 1) > ndev:
            # ranks share a GPU (rehearsals): the one-launch BatchNorm needs its whole grid co-resident, which
            # another process's kernels on the same CUs can prevent (its bounded wait then reports a timeout,
            # ops.functional.check_device_errors) -- use the multi-launch BatchNorm instead
            os.environ.setdefault("PDE_BN_FUSED", "0")
    else:
        dev = torch.device("cpu")
    if backend == "gloo" and os.environ.get("MASTER_ADDR", "127.0.0.1") in ("127.0.0.1", "localhost"):
        # single-host gloo: bind the loopback device explicitly (the container hostname may not resolve,
        # which otherwise makes re-formed groups after a torchrun restart fail to connect)
        os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
    if not dist.is_initialized():
        if init_method is None:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if "MASTER_PORT" not in os.environ:
                if world_size != 1:
                    raise RuntimeError("MASTER_PORT must be set for a multi-process job")
                os.environ["MASTER_PORT"] = str(free_port())
            init_method = "env://"
        kw = dict(backend=backend, init_method=init_method, rank=rank, world_size=world_size,
                  timeout=datetime.timedelta(seconds=timeout_s))
        if (init_method == "env://" and os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True"
                and "TORCHELASTIC_RESTART_COUNT" in os.environ):
            # torchrun restarts reuse the agent's TCPStore (same MASTER_PORT), and torch's env:// handler adds
            # no per-attempt prefix: a restarted rank could read the PREVIOUS attempt's gloo / RCCL rendezvous
            # keys of a dead peer ("Connection refused", then a hang in connectFullMesh -- measured on this
            # container, ~1 restart in 4).  Every attempt gets its own key space.
            store = dist.TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]), world_size,
                                  is_master=False, timeout=kw["timeout"])
            kw.pop("init_method")
            kw["store"] = dist.PrefixStore(f"/pde/attempt_{os.environ['TORCHELASTIC_RESTART_COUNT']}", store)
        if backend == "nccl" and use_gpu:
            kw["device_id"] = dev
        dist.init_process_group(**kw)
    return DistContext(rank, world_size, local_rank, dev, backend)


def shutdown() -> None:
    if dist.is_initialized():
        dist.destroy_process_group()


def world() -> int:
    return dist.get_world_size() if dist.is_initialized() else 1


def rank() -> int:
    return dist.get_rank() if dist.is_initialized() else 0


def barrier(ctx: DistContext | None = None) -> None:
    if dist.is_initialized() and dist.get_world_size() > 1:
        if ctx is not None and ctx.device.type == "cuda":
            dist.barrier(device_ids=[ctx.device.index])
        else:
            dist.barrier()


def max_over_ranks(value: float, device) -> float:
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value: float, device) -> float:
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())
