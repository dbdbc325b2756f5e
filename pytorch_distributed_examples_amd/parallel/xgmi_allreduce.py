"""One-shot xGMI peer all-reduce for latency-bound buckets, and the DDP communicator that routes buckets
between it and RCCL (SURVEY.md §5.8 items 2-3, §7.1 ``xgmi_allreduce.hip``).

Why: the MNIST CNN reduces one 87 KB gradient bucket per 50 us step (horovod/mnist_horovod.py:53 is a
per-step all-reduce; rpc/server_model_data_parallel.py:41 a 544 B one).  A ring all-reduce of that size is
2(N-1) dependent latency-bound hops; on a fully connected MI355X node every rank can instead read all 7
peers' buckets directly over their 7 xGMI links and reduce locally: one kernel, one flag exchange
(csrc/comm/xgmi_allreduce.hip).  Large buckets stay on RCCL, whose multi-channel rings/trees use the links'
bandwidth better than 7 full copies per rank.

    xa = XgmiAllreduce(device)            # collective: exchanges IPC handles through the c10d store
    xa.allreduce_(grads, avg=True)        # stream-ordered, hipGraph-capturable, bit-identical on all ranks
    fused.forward_backward(x, y, sgd=opt, xgmi=xa)   # the CNN folds the exchange into its reduction kernel
    comm = RoutedComm(StreamComm(device), xa, threshold_bytes=1 << 20)
    ddp = DistributedDataParallel(model, comm=comm)

On one GPU the same code runs with several processes sharing the card (the IPC mapping then points back
at the same device), which is how the protocol is rehearsed on single-GPU boxes.
"""
from __future__ import annotations

import itertools
import os

import torch
import torch.distributed as dist

from .. import _native

_SEQ = itertools.count()
DEFAULT_THRESHOLD = int(os.environ.get("PDE_XGMI_THRESHOLD", str(1 << 20)))


class XgmiAllreduce:
    """``two_shot=True``: the bandwidth form (reduce-scatter + all-gather through the same IPC slots,
    ``XgmiAllreduce::allreduce_twoshot``): each rank reduces 1/N of the bucket from all peers and the others read that
    sum back, so every xGMI link carries 2/N of the bucket instead of all of it -- for large buckets (a pipeline
    stage's 24M gradients).  An instance runs one form only."""

    def __init__(self, device: torch.device, group=None, max_bytes: int = 4 << 20, blocks: int = 256,
                 timeout_s: float | None = None, read_delay_us: float = 0.0, key: str | None = None,
                 two_shot: bool = False):
        if timeout_s is None:  # PDE_XGMI_TIMEOUT_S: the bounded peer wait (seconds)
            timeout_s = float(os.environ.get("PDE_XGMI_TIMEOUT_S", "5.0"))
        assert device.type == "cuda", "the xGMI all-reduce is a GPU data plane"
        self.device = device
        self.two_shot = bool(two_shot)
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.size = dist.get_world_size(group) if dist.is_initialized() else 1
        C = _native.comm()
        self.impl = C.XgmiAllreduce(self.rank, self.size, device.index, int(max_bytes), int(blocks), float(timeout_s))
        if read_delay_us:  # test hook: a slow reader (tests/test_xgmi_gpu.py)
            self.impl.set_read_delay_us(float(read_delay_us))
        if self.size > 1:
            store = dist.distributed_c10d._get_default_store()
            ranks = dist.get_process_group_ranks(group) if group is not None else list(range(self.size))
            # ``key``: an explicit handshake key (members that joined at different times -- an elastic
            # round -- have different local counters)
            key = (f"pde/xgmi{'2' if two_shot else ''}/{key if key is not None else next(_SEQ)}/"
                   f"{'-'.join(map(str, ranks))}")
            store.set(f"{key}/{self.rank}", self.impl.ipc_handle())
            handles = [store.get(f"{key}/{r}") for r in range(self.size)]
            self.impl.open(handles)

    @property
    def max_bytes(self) -> int:
        return self.impl.max_bytes

    def allreduce_(self, t: torch.Tensor, avg: bool = False, wire_bf16: bool = False) -> torch.Tensor:
        """In-place fp32 all-reduce; ``wire_bf16``: peers exchange bf16 copies (cast fused into the staging,
        half the xGMI bytes), the sum and the result stay fp32."""
        if self.two_shot:
            self.impl.allreduce_twoshot_(t, 1.0 / self.size if avg else 1.0, wire_bf16)
        else:
            self.impl.allreduce_(t, 1.0 / self.size if avg else 1.0, wire_bf16)
        return t

    def view(self) -> list:
        """Flat device view (csrc/comm/xgmi_view.h) for kernels that fold the exchange into their own
        epilogue: the fused CNN's gradient reduction (``FusedCNN.forward_backward(..., xgmi=self)``)."""
        return self.impl.view()

    def check(self, clear: bool = True) -> None:
        """Raise if any call timed out waiting for a peer (or gave up on ``abort()``); synchronises the
        device.  ``clear``: reset the error words first, so the instance is usable again once the caller has
        handled the failure (re-synced the replicas) -- the device-side fail-fast word would otherwise make
        every later call drop its result."""
        if self.impl.error(True):
            if clear:
                self.impl.clear_error()
            raise RuntimeError("xGMI all-reduce: a workgroup timed out waiting for a peer's flag")

    def failed(self) -> bool:
        """Non-blocking: True once a queued call has timed out (a plain read of the host-mapped status word;
        calls still in flight are not waited for).  Cheap enough for every step."""
        return bool(self.impl.error(False))

    def abort(self) -> None:
        """Make every spinning and later peer wait give up at once (from any thread; e.g. the elastic
        membership watcher when the driver publishes a new round)."""
        self.impl.abort()

    def reset_abort(self) -> None:
        self.impl.reset_abort()

    def close(self):
        if self.impl is not None:
            self.impl.close()
            self.impl = None


class _Done:
    def wait(self):
        return True

    def is_completed(self):
        return True


class RoutedComm:
    """DDP communicator plug-in (``size``, ``rank``, ``supports_avg``, ``allreduce_async``, ``broadcast_``):
    fp32 buckets up to ``threshold_bytes`` take the one-shot xGMI path; larger fp32 buckets up to the two-shot
    instance's ``max_bytes`` take the two-shot xGMI path (``xgmi2``, single-node jobs; ``PDE_XGMI_TWOSHOT=0``: RCCL);
    the rest (and non-fp32 tensors) go to RCCL.  ``rccl=None`` (ranks sharing one GPU: RCCL refuses duplicate
    devices): every bucket takes an xGMI path and must fit ``xgmi2.max_bytes``."""

    def __init__(self, rccl, xgmi: XgmiAllreduce, threshold_bytes: int = DEFAULT_THRESHOLD, xgmi2=None):
        self.rccl, self.xgmi, self.xgmi2 = rccl, xgmi, xgmi2
        self.size, self.rank = xgmi.size, xgmi.rank
        self.supports_avg = True
        self.threshold = min(int(threshold_bytes), xgmi.max_bytes)
        self.routed = {"xgmi": 0, "xgmi2": 0, "rccl": 0}
        self._scratch: dict = {}  # persistent bf16 wire buffers of RCCL-routed fp32 tensors

    def _two_shot(self, t: torch.Tensor) -> bool:
        return (self.xgmi2 is not None and t.dtype == torch.float32 and t.is_contiguous()
                and t.numel() * 4 <= self.xgmi2.max_bytes)

    def fuses_bf16_wire(self, t: torch.Tensor) -> bool:
        """True when ``allreduce_async(t, wire_bf16=True)`` casts inside the one-shot kernel (the bucket
        takes the xGMI path); DDP casts larger buckets itself into persistent bf16 buffers for RCCL."""
        return t.dtype == torch.float32 and (t.numel() * 4 <= self.threshold or self._two_shot(t))

    def allreduce_async(self, t: torch.Tensor, avg: bool = False, wire_bf16: bool = False):
        """``wire_bf16`` (fp32 ``t``): reduce bf16 copies -- fused into the one-shot kernel on the xGMI path;
        on RCCL our cast kernels into / out of a persistent bf16 scratch around a bf16 all-reduce."""
        if t.dtype == torch.float32 and t.numel() * 4 <= self.threshold:
            self.xgmi.allreduce_(t, avg, wire_bf16)
            self.routed["xgmi"] += 1
            return _Done()
        if self._two_shot(t):
            self.xgmi2.allreduce_(t, avg, wire_bf16)
            self.routed["xgmi2"] += 1
            return _Done()
        if self.rccl is None:
            raise RuntimeError(f"xGMI-only communicator: a {t.dtype} bucket of {t.numel()} elements fits no xGMI path")
        self.routed["rccl"] += 1
        if wire_bf16 and t.dtype == torch.float32:
            C = _native.C()
            key = (t.data_ptr(), t.numel())
            w = self._scratch.get(key)
            if w is None:
                w = self._scratch[key] = torch.empty(t.numel(), dtype=torch.bfloat16, device=t.device)
            C.cast_bf16_into(t.reshape(-1), w)
            self.rccl.allreduce_async(w, avg)
            C.cast_f32_into(w, t.reshape(-1))  # stream-ordered behind the collective
            return _Done()
        return self.rccl.allreduce_async(t, avg)

    def allreduce_(self, t: torch.Tensor, avg: bool = False) -> torch.Tensor:
        self.allreduce_async(t, avg)
        return t

    def check(self) -> None:
        """Raise if an xGMI exchange timed out (its result was dropped); synchronises the device -- call
        it at existing sync points (epoch end, before snapshots)."""
        self.xgmi.check()
        if self.xgmi2 is not None:
            self.xgmi2.check()

    def broadcast_(self, t: torch.Tensor, src: int) -> torch.Tensor:
        if self.rccl is not None:
            return self.rccl.broadcast_(t, src)
        # xGMI only: a broadcast is the sum of src's tensor and everyone else's zeros (exact in fp32), chunked
        # through the two-shot instance (construction time only: parameters and buffers)
        flat = t.reshape(-1)
        work = flat.float() if flat.dtype != torch.float32 else flat.clone()
        if self.rank != src:
            work.zero_()
        inst = self.xgmi2 if self.xgmi2 is not None else self.xgmi
        step = inst.max_bytes // 4
        for s0 in range(0, work.numel(), step):
            inst.allreduce_(work[s0:s0 + step], False)  # (1-D slices of a contiguous tensor: in place)
        with torch.no_grad():
            t.copy_(work.view_as(t).to(t.dtype))
        return t

    def destroy(self):
        self.xgmi.close()
        if self.xgmi2 is not None:
            self.xgmi2.close()
        if self.rccl is not None:
            self.rccl.destroy()


def xgmi_only_comm(device: torch.device, group=None, max_bytes: int = 64 << 20, key: str | None = None) -> RoutedComm:
    """A DDP communicator without RCCL: one-shot xGMI for small buckets, two-shot for the rest (buckets up to
    ``max_bytes``).  It runs with several ranks sharing one GPU, which is how a pipeline x data-parallel job is
    rehearsed on a one-GPU box (RCCL refuses two ranks on one device); on a node it is a pure-IPC data plane."""
    # the peer-wait bound: ranks sharing one GPU (the rehearsal) start far apart on their first step (every
    # process loads its code objects at once), so the default here is generous (PDE_XGMI_TIMEOUT_S overrides)
    t = float(os.environ.get("PDE_XGMI_TIMEOUT_S", "60"))
    shared = torch.cuda.device_count() < int(os.environ.get("LOCAL_WORLD_SIZE", "1"))
    small = XgmiAllreduce(device, group=group, key=None if key is None else key + "/1", timeout_s=t,
                          blocks=8 if shared else 256)
    # two-shot workgroups.  Ranks sharing ONE GPU (the rehearsal): a few -- a 256-workgroup grid spinning on its
    # DP peer starves the other processes' kernels on the card (profiles/r6f: the other pipeline made no progress
    # until the wait timed out; 8 or 1 workgroups: every step and graph replay completes).  A node: 256.
    blocks = int(os.environ.get("PDE_XGMI2_BLOCKS", "8" if shared else "256"))
    big = XgmiAllreduce(device, group=group, max_bytes=max_bytes, blocks=blocks, two_shot=True,
                        key=None if key is None else key + "/2", timeout_s=t)
    return RoutedComm(None, small, xgmi2=big)
