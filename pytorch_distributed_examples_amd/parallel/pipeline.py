"""Intra-node pipeline parallelism over xGMI.

Replaces the reference's RPC data path (rpc/model_parallel_ResNet50.py:167-178: every micro-batch is
pulled with ``RRef.to_here()`` as a CPU tensor, three process hops per micro-batch) with a
stage-per-GPU engine:

* activations and activation-gradients stay in HBM and move GPU->GPU over the one direct xGMI link of a
  neighbouring stage pair: by default through an IPC-mapped receive ring that the sender's kernel writes
  directly (csrc/comm/p2p_ring.hip: epoch flags, credits, bounded spins -- and rehearsable with two
  processes on ONE GPU), or with ``PDE_P2P=rccl`` RCCL ``send``/``recv`` on dedicated 2-rank
  communicators; stream-ordered with the producing kernels either way (no host synchronisation, no
  ``.cpu()``, quirk Q13 fixed), so a whole pipelined step records into one hipGraph;
* stage boundaries carry bf16 NHWC activations (ResNet-50 at the layer2|layer3 cut: m x 16 x 16 x 512,
  4x fewer bytes than the reference's fp32 tensors);
* explicit schedules: ``gpipe`` (all forwards, then all backwards -- the reference's fill/drain) and
  ``1f1b`` (steady-state one-forward-one-backward; same bubble, bounded in-flight activations);
* per-micro-batch BatchNorm statistics (quirk Q17 kept), also when several micro-batches run as one
  pipeline unit (``bn_groups``): at micro-batch 4-8 every ResNet-50 kernel is latency-bound on MI355X
  (stage 1: 1.11 ms at m = 8 vs 1.68 ms at m = 32, profiles/r3f_stage_bench.jsonl), so a stage runs G
  micro-batches per launch sequence with grouped BatchNorm -- the reference's math at 1/G of the launches;
* composes with data parallelism: ``dp_group`` all-reduces each stage's gradients across its replicas
  (hybrid "2-stage pipeline x 4-way DDP" of BASELINE config 4).

The engine is SPMD: every stage process calls ``train_step``; stage 0 feeds inputs, the last stage
owns targets and the loss.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from .. import _native
from ..ops import functional as OF
from ..utils.log import NO_PHASES


def p2p_mode(device: torch.device) -> str:
    """Data plane of the stage channels: ``ring`` (IPC receive ring over xGMI, default on GPUs), ``rccl``
    (RCCL send/recv; needs the nccl backend) or ``host`` (gloo through host memory: CPU, or forced)."""
    if device.type != "cuda":
        return "host"
    mode = os.environ.get("PDE_P2P", "ring")
    if mode == "rccl" and dist.get_backend() != "nccl":
        return "host"
    return mode if mode in ("ring", "rccl", "host") else "ring"


class P2PChannel:
    """Point-to-point channel between two neighbouring stage processes (ranks lo < hi of the default group).

    GPU data plane, ``ring`` (default): each side exports one IPC-mapped receive ring in its HBM
    (csrc/comm/p2p_ring.hip); ``send`` is ONE kernel that writes the tensor straight into the peer's ring
    slot over xGMI and raises per-workgroup flags there, ``recv`` is ONE kernel that waits for them, copies
    the slot into a fresh tensor and returns a credit to the sender.  Sequence numbers live on the device,
    so the kernels are capturable and every hipGraph replay moves the next messages.  Two processes on one
    GPU map each other's rings exactly like two GPUs of a node: the pipeline data plane is rehearsed on
    single-GPU boxes (tests/test_pipeline_gpu.py).

    ``rccl``: TWO 2-rank RCCL communicators, one per direction -- ``down`` carries lo -> hi traffic
    (activations), ``up`` carries hi -> lo traffic (activation gradients).  RCCL executes the operations
    of one communicator in issue order whatever stream they are enqueued on, so with a single
    communicator the 1F1B steady state (stage 0: send a1, recv g0; stage 1: send g0, recv a1) would pair
    a send with a send and deadlock.  With one communicator per direction every communicator only ever
    sees send on one side and recv on the other, in the same order.  Unique ids go through the default
    store.

    Either way ``send``/``recv`` are stream-ordered (capturable into a hipGraph, no host synchronisation);
    sends run on a dedicated side stream so the compute stream never waits for the peer.

    CPU configuration (``host``): gloo ``isend``/``recv`` with one tag per direction; device tensors are
    staged through host memory."""

    TAG_DOWN, TAG_UP = 11, 12

    def __init__(self, peer: int, tag: str, device: torch.device, store=None):
        me = dist.get_rank()
        self.peer = peer
        self.lo, self.hi = min(me, peer), max(me, peer)
        self.local_rank = 0 if me == self.lo else 1
        self.peer_local = 1 - self.local_rank
        self.device = device
        self.down = self.up = None
        self.ring = None
        self._meta = {}
        self._pending = []
        self._inflight = []  # tensors sent on the side stream: kept alive until flush() joins the streams
        self._send_stream = None
        self.mode = p2p_mode(device)
        self.rccl = self.mode == "rccl"
        self._store = store or (dist.distributed_c10d._get_default_store() if self.mode != "host" else None)
        self._key = f"pde/p2p/{tag}/{self.lo}-{self.hi}"
        if self.mode == "ring":
            C = _native.comm()
            slot = int(float(os.environ.get("PDE_P2P_SLOT_MB", "16")) * (1 << 20))
            self.ring = C.P2PRing(device.index, slot, float(os.environ.get("PDE_P2P_TIMEOUT_S", "60")))
            self._store.set(f"{self._key}/ring/{self.local_rank}", self.ring.ipc_handle())
            self.ring.open(self._store.get(f"{self._key}/ring/{self.peer_local}"))
            # sends wait for credit on a side stream with their whole grid resident: keep that many CUs out of
            # the one-launch BatchNorm's co-residency budget
            from ..ops.functional import BnHeadroom

            self._bn_headroom = BnHeadroom(C.P2PRing.max_wg())
            return
        if not self.rccl:
            return
        store = self._store
        C = _native.comm()
        comms = []
        for direction in ("down", "up"):  # same creation order on both ranks
            key = f"{self._key}/{direction}"
            if self.local_rank == 0:
                store.set(key, C.rccl_unique_id())
            uid = store.get(key)
            c = C.RcclComm()
            c.init(uid, self.local_rank, 2, device.index, True)
            comms.append(c)
        self.down, self.up = comms

    # direction of a send/recv from this rank's point of view
    def _send_comm(self):
        return self.down if self.local_rank == 0 else self.up

    def _recv_comm(self):
        return self.up if self.local_rank == 0 else self.down

    def _tag(self, sending: bool) -> int:
        lo_side = self.local_rank == 0
        return self.TAG_DOWN if (lo_side == sending) else self.TAG_UP

    def _gpu_send(self, t: torch.Tensor):
        if self.ring is not None:
            if t.data_ptr() % 16:  # the ring kernel copies 16-B vectors
                t = t.clone()
            self.ring.send(t)  # slot-sized pieces for large tensors (p2p_ring.hip)
        else:
            self._send_comm().send(t, self.peer_local)

    def send(self, t: torch.Tensor):
        """Asynchronous send.  GPU: enqueued on a dedicated send stream (after the producer's work), so
        the compute stream never waits for the peer to post its receive.  host: isend, completed in
        :meth:`flush`."""
        t = t.contiguous()
        if self.mode == "host":
            src = t.cpu() if t.is_cuda else t
            self._pending.append((dist.isend(src, self.peer, tag=self._tag(True)), src))
            return
        if self._send_stream is None:
            # high priority: sends spin waiting for the peer's credit; on a hardware queue shared with the compute
            # stream they would hold back the compute stream's own receives (a cross-rank wait cycle in 1F1B)
            self._send_stream = torch.cuda.Stream(device=self.device, priority=-1)
        cur = torch.cuda.current_stream(self.device)
        self._send_stream.wait_stream(cur)
        with torch.cuda.stream(self._send_stream):
            self._gpu_send(t)
        if torch.cuda.is_current_stream_capturing():
            # inside a hipGraph capture: no allocator stream bookkeeping; the tensor stays referenced
            # until flush() has joined the send stream back into the capturing stream
            self._inflight.append(t)
        else:
            t.record_stream(self._send_stream)

    def flush(self):
        """Complete outstanding sends (host) / order the compute stream after them (GPU)."""
        for work, _ in self._pending:
            work.wait()
        self._pending = []
        if self._send_stream is not None:
            torch.cuda.current_stream(self.device).wait_stream(self._send_stream)
        self._inflight = []

    def recv(self, shape, dtype) -> torch.Tensor:
        t = torch.empty(shape, dtype=dtype, device=self.device)
        if self.mode == "host":
            if t.is_cuda:
                h = torch.empty(shape, dtype=dtype)
                dist.recv(h, self.peer, tag=self._tag(False))
                t.copy_(h)
            else:
                dist.recv(t, self.peer, tag=self._tag(False))
        elif self.ring is not None:
            self.ring.recv(t)
        else:
            self._recv_comm().recv(t, self.peer_local)
        return t

    def check(self):
        """Raise if a ring wait timed out (synchronises the device)."""
        if self.ring is not None and self.ring.error():
            raise RuntimeError(f"p2p ring {self._key}: a send/recv timed out waiting for the peer")

    def send_meta(self, t: torch.Tensor):
        """Shape/dtype handshake (first micro-batch only), 8 int64s over the same channel."""
        codes = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}
        m = torch.zeros(8, dtype=torch.long, device=self.device)
        m[0] = t.dim()
        m[1] = codes[t.dtype]
        m[2:2 + t.dim()] = torch.tensor(list(t.shape), dtype=torch.long)
        self.send(m)

    def recv_meta(self):
        m = self.recv((8,), torch.long).cpu().tolist()
        dtype = {0: torch.float32, 1: torch.bfloat16, 2: torch.float16}[m[1]]
        return tuple(m[2:2 + m[0]]), dtype

    def close(self):
        for c in (self.down, self.up):
            if c is not None:
                c.destroy()
        self.down = self.up = None
        if self.ring is not None:
            # the peer writes into my ring and ACKs into my ctrl word: both sides drain, meet, then unmap
            torch.cuda.synchronize(self.device)
            self._store.set(f"{self._key}/closed/{self.local_rank}", "1")
            self._store.get(f"{self._key}/closed/{self.peer_local}")
            self.ring.close()
            self.ring = None
            if getattr(self, "_bn_headroom", None) is not None:
                self._bn_headroom.release()


class PipelineEngine:
    def __init__(self, module: torch.nn.Module, stage: int, num_stages: int, prev_rank: int | None,
                 next_rank: int | None, device: torch.device, loss_fn=None, schedule: str = "gpipe",
                 tag: str = "pipe"):
        assert schedule in ("gpipe", "1f1b")
        self.module = module
        self.stage, self.num_stages = stage, num_stages
        self.first, self.last = stage == 0, stage == num_stages - 1
        self.device = device
        self.loss_fn = loss_fn
        self.schedule = schedule
        # channels are created in a fixed global order (lower rank pair first) to avoid init deadlocks
        self.prev = self.next = None
        pairs = []
        if prev_rank is not None:
            pairs.append(("prev", prev_rank))
        if next_rank is not None:
            pairs.append(("next", next_rank))
        for which, peer in sorted(pairs, key=lambda p: min(p[1], dist.get_rank())):
            ch = P2PChannel(peer, tag, device)
            setattr(self, which, ch)
        self._fwd_meta = None  # (shape, dtype) of activations received from prev
        self._unit = None
        self._bwd_meta = None
        self.timer = NO_PHASES  # utils.log.PhaseTimer: per-stage fwd / bwd / recv-wait times (bench)
        # micro-batches per pipeline unit: each unit passed to train_step is `bn_groups` micro-batches run as
        # ONE launch sequence with per-micro-batch BatchNorm statistics (ops.functional.bn_groups)
        self.bn_groups = 1
        # a DistributedDataParallel(overlap=True) over this stage's replicas: its bucket all-reduces fire
        # during the LAST micro-batch's backward (earlier ones run under no_sync), overlapping the rest of it
        self.ddp = None

    # -- primitives --------------------------------------------------------------------------------
    def _recv_act(self):
        if self._fwd_meta is None:
            self._fwd_meta = self.prev.recv_meta()
        x = self.prev.recv(*self._fwd_meta)
        return x.requires_grad_(True)

    def _send_act(self, y, first_mb):
        if first_mb and not getattr(self, "_sent_meta", False):
            self.next.send_meta(y)
            self._sent_meta = True
        self.next.send(y.detach())

    def _forward(self, mb, inputs, targets, n_mb, state):
        if self.first:
            x = inputs[mb]
        else:
            with self.timer.phase("recv_wait"):
                x = self._recv_act()
        with self.timer.phase("fwd"), OF.bn_groups(self.bn_groups):
            y = self.module(x)
            loss = self.loss_fn(y, targets[mb]) / n_mb if self.last else None
        if self.last:
            state["loss"].append(loss.detach())
            state["saved"][mb] = (x, loss, None)
        else:
            self._send_act(y, mb == 0)
            state["saved"][mb] = (x, y, None)

    def _backward(self, mb, state):
        if self.ddp is not None and mb != state["n_mb"] - 1:
            with self.ddp.no_sync():
                return self._backward_mb(mb, state)
        return self._backward_mb(mb, state)

    def _backward_mb(self, mb, state):
        x, y, _ = state["saved"].pop(mb)
        if self.last:
            with self.timer.phase("bwd"):
                if self._unit is None or self._unit.shape != y.shape or self._unit.dtype != y.dtype:
                    self._unit = torch.ones_like(y)  # persistent d loss = 1: no fill kernel per micro-batch
                y.backward(self._unit)
        else:
            with self.timer.phase("recv_wait"):
                g = self.next.recv(y.shape, y.dtype)
            with self.timer.phase("bwd"):
                torch.autograd.backward(y, g)
        if not self.first:
            self.prev.send(x.grad)

    # -- schedules --------------------------------------------------------------------------------
    def train_step(self, inputs=None, targets=None, num_microbatches: int = 1):
        """One pipelined forward+backward over ``num_microbatches``; returns the loss (last stage) or
        None.  ``inputs``/``targets`` are lists of micro-batches (stage 0 / last stage)."""
        M = num_microbatches
        st = {"saved": {}, "loss": [], "n_mb": M}
        if self.schedule == "gpipe":
            for mb in range(M):
                self._forward(mb, inputs, targets, M, st)
            for mb in range(M):
                self._backward(mb, st)
        else:  # 1F1B
            warm = min(M, self.num_stages - self.stage - 1)
            f = b = 0
            for _ in range(warm):
                self._forward(f, inputs, targets, M, st)
                f += 1
            while f < M:
                self._forward(f, inputs, targets, M, st)
                f += 1
                self._backward(b, st)
                b += 1
            while b < M:
                self._backward(b, st)
                b += 1
        for ch in (self.prev, self.next):
            if ch is not None:
                ch.flush()
        if self.last:
            return torch.stack(st["loss"]).sum()
        return None

    @torch.no_grad()
    def forward_only(self, inputs=None, num_microbatches: int = 1):
        outs = []
        for mb in range(num_microbatches):
            x = inputs[mb] if self.first else self.prev.recv(*self._meta_or_handshake())
            y = self.module(x)
            if self.last:
                outs.append(y)
            else:
                self._send_act(y, mb == 0)
        return torch.cat(outs) if outs else None

    def _meta_or_handshake(self):
        if self._fwd_meta is None:
            self._fwd_meta = self.prev.recv_meta()
        return self._fwd_meta

    def check(self):
        """Raise if a ring wait or a one-launch BatchNorm hand-off of this stage timed out (syncs the device)."""
        for ch in (self.prev, self.next):
            if ch is not None:
                ch.check()
        if self.device.type == "cuda":
            OF.check_device_errors(f"pipeline stage {self.stage}")

    def close(self):
        for ch in (self.prev, self.next):
            if ch is not None:
                ch.close()


def hybrid_groups(world: int, stages: int):
    """Rank layout for ``stages``-deep pipelines x ``world // stages`` data-parallel replicas.

    Pipelines are consecutive ranks (0,1), (2,3), ... -- on an MI355X node every pair is one direct xGMI
    link; DP groups are ranks with the same stage index ({0,2,4,6} and {1,3,5,7} at world 8).
    Returns (pipelines, dp_groups) as lists of rank lists."""
    assert world % stages == 0
    pipes = [list(range(p * stages, (p + 1) * stages)) for p in range(world // stages)]
    dps = [[p[s] for p in pipes] for s in range(stages)]
    return pipes, dps
