"""In-process communicator re-wire for elastic DDP (SURVEY.md P3 / §5.3 "re-wire RCCL without a job
restart").

The reference's elastic DDP (pytorch_elastic/mnist_ddp_elastic.py, launched by torchrun ``--max-restarts``)
survives a failure by killing and restarting EVERY worker, which then reload ``snapshot.pt``
(mnist_ddp_elastic.py:54-56; observed in SURVEY.md §5.3).  ``mnist_ddp_elastic.py --rewire`` instead keeps
the surviving processes -- and their device-resident model, optimizer state and data -- alive:

1. workers are launched by the elastic driver (:mod:`..launch.hvdrun`), which publishes membership
   *rounds* in a TCPStore (:mod:`.rendezvous`);
2. each round gets a fresh gloo control group and, on GPUs, a fresh RCCL communicator of our own
   (:class:`_comm.RcclComm`, unique id in the round's ``PrefixStore``), which DDP uses for its buckets;
3. a dead peer surfaces as a failed gloo collective (CPU) or as an RCCL collective that does not finish
   while the driver has already published a newer round (GPU): the communicator is ``ncclCommAbort``-ed,
   the survivors restore their last in-memory commit and join the next round;
4. workers added by host discovery are picked up at the next commit point: all ranks agree on the
   driver's ``updated`` flag (MAX all-reduce), close the round cleanly and re-join together;
5. after every (re)join rank 0 -- always a survivor holding the newest commit -- broadcasts model,
   optimizer state and the epoch position; the sampler is re-sharded for the new world size and resumes
   at the first batch not yet consumed by the whole group.

Commits are device-resident clones (one D2D copy per tensor, 288 GB of HBM leaves plenty of room).
"""
from __future__ import annotations

import datetime
import os
import time

import torch
import torch.distributed as dist

from .. import _native
from . import fault
from ..utils.state import clone_state as _clone
from .rendezvous import RendezvousClient


class PeerFailure(RuntimeError):
    """A collective of the current round failed (a member died or hung)."""


class MembershipChanged(Exception):
    """The driver published a new round (hosts added/removed); re-join at a commit point."""


class _CpuWork:
    def __init__(self, work):
        self.work = work

    def wait(self):
        try:
            self.work.wait()
        except RuntimeError as exc:
            raise PeerFailure(str(exc)) from exc


class _GpuWork:
    """An RCCL bucket all-reduce on the current stream.  ``wait()`` does not block the host: everything
    that consumes the bucket is stream-ordered behind the collective.  Liveness is checked once per step
    instead (:meth:`RoundComm.step_done`, one step behind) and at commit points (:meth:`RoundComm.drain`)."""

    def __init__(self, comm, event):
        self.comm, self.event = comm, event

    def wait(self):
        return True


def _emulated() -> bool:
    """``PDE_REWIRE_EMULATE=gloo``: on CPU, RoundComm's data-plane communicator is a gloo stand-in for RCCL
    (:class:`..parallel.gloo_comm.GlooComm`) so the init / shrink / split protocol runs in the CPU tests."""
    return os.environ.get("PDE_REWIRE_EMULATE", "") == "gloo"


class RoundComm:
    """Communicator set of one rendezvous round (see the module docstring).

    How the round's RCCL communicator is built (``self.how``), agreed by every member over the round's gloo
    group first so no member can take a different path:

    * ``split`` -- a PLANNED scale-down (the driver dropped hosts; every old member alive): all members of the
      previous round called :meth:`planned_split` at its last commit point (``ncclCommSplit``, the leavers
      with ``NCCL_SPLIT_NOCOLOR``) and pass the child here as ``premade``: no unique-id exchange, topology
      reused (ref: horovod/horovod_mnist_elastic.py:108 ``--min-np`` shrink);
    * ``shrink`` -- after a FAILURE, when this round only drops members of ``parent``'s round (same order), the
      parent's communicator is still valid on EVERY survivor and the loaded RCCL exports ``ncclCommShrink``
      (torch's bundled RCCL 2.26 does not);
    * ``init`` -- otherwise: a fresh communicator from a new unique id (growth, or a shrink RCCL cannot do).

    ``use_rccl=False``: control plane only (the fused CNN exchanges gradients over xGMI inside its reduction
    kernel).  ``timing`` holds the seconds spent on the control group and on the data-plane communicator."""

    emulated = False  # gloo stand-in for RCCL (PDE_REWIRE_EMULATE=gloo, CPU only)

    def __init__(self, rdzv: RendezvousClient, rank: int, size: int, device: torch.device,
                 timeout_s: float = 120.0, grace_s: float = 2.0, parent: "RoundComm | None" = None,
                 use_rccl: bool = True, premade=None):
        self.rdzv, self.rank, self.size, self.device = rdzv, rank, size, device
        self.timeout_s, self.grace_s = timeout_s, grace_s
        self.members = rdzv.members()
        self.how = "none"
        self.timing = {}
        t0 = time.perf_counter()
        store = rdzv.pg_store()
        dist.init_process_group("gloo", store=store, rank=rank, world_size=size,
                                timeout=datetime.timedelta(seconds=timeout_s))
        t1 = time.perf_counter()
        self.timing["control_group_s"] = t1 - t0
        self.rccl = None
        self.emulated = device.type == "cpu" and _emulated()
        if use_rccl and size > 1 and (device.type == "cuda" or self.emulated):
            self._build_data_plane(store, parent, premade)
        elif premade is not None:
            premade[1].abort()  # a one-rank round needs no data plane
        if parent is not None:
            parent.release()
        self.timing["data_plane_s"] = time.perf_counter() - t1
        self.supports_avg = self.rccl is not None
        self._steps = []  # end-of-step events not yet checked on the host (GPU data plane)

    def _comm_cls(self):
        if self.emulated:
            from ..parallel.gloo_comm import GlooComm

            return GlooComm
        return _native.comm().RcclComm

    def _build_data_plane(self, store, parent, premade):
        Comm = self._comm_cls()
        excl = self._shrink_plan(parent)
        code = 0
        if premade is not None and premade[0] == self.members and premade[1].valid:
            code = 2
        elif excl is not None and Comm.shrink_supported():
            code = 1
        t = torch.tensor([float(code), -float(code)])
        try:
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
        except RuntimeError as exc:
            raise PeerFailure(str(exc)) from exc
        lo, hi = int(t[0].item()), int(-t[1].item())
        if lo == 2:
            self.rccl, self.how = premade[1], "split"
            return
        if premade is not None:
            premade[1].abort()
        if lo == 1 and hi == 1:
            self.rccl = Comm()
            self.rccl.shrink_from(parent.rccl, excl, True)
            self.how = "shrink"
            return
        self.rccl = Comm()
        if self.emulated:
            self.rccl.init(store, "emu_rccl", self.rank, self.size, self.timeout_s)
        else:
            if self.rank == 0:
                store.set("rccl_uid", _native.comm().rccl_unique_id())
            uid = store.get("rccl_uid")
            self.rccl.init(uid, self.rank, self.size, self.device.index, True)
        self.how = "init"

    def _shrink_plan(self, parent):
        """Parent ranks to exclude when this round only drops members of the parent's round and the parent's
        communicator is still valid HERE, else None (a PeerFailure usually aborted it already)."""
        if parent is None or parent.rccl is None or not parent.rccl.valid or not parent.members or not self.members:
            return None
        if not set(self.members) < set(parent.members):
            return None
        survivors = [m for m in parent.members if m in self.members]
        if survivors != self.members:  # the shrunk communicator keeps the parent's rank order
            return None
        return [i for i, m in enumerate(parent.members) if m not in self.members]

    def planned_split(self):
        """Collective over THIS round (every member alive, at a commit point that raised MembershipChanged):
        when the driver's newest round keeps a subset of this round's members in the same order, split the
        RCCL communicator for it (``ncclCommSplit``; leavers pass NOCOLOR).  Returns ``("leave", None)`` for a
        worker the newest round no longer contains, ``("split", (members, child))`` for a survivor of a split,
        else ``("none", None)`` (growth or reordering: the next round initialises)."""
        rdzv = self.rdzv
        newest = None
        if self.rank == 0:
            deadline = time.time() + 30.0
            while rdzv._current_round() <= rdzv.round and time.time() < deadline:
                time.sleep(0.02)
            newest = rdzv._current_round()
        newest = self.broadcast_object(newest) if self.size > 1 else newest
        members = rdzv.members(newest) if newest is not None and newest > rdzv.round else []
        leaving = bool(members) and rdzv.wid not in members
        subset = bool(members) and set(members) < set(self.members) and \
            [m for m in self.members if m in members] == members
        if not subset or self.rccl is None or not self.rccl.valid:
            return ("leave", None) if leaving else ("none", None)
        child = self._comm_cls()()
        try:
            # bounded by the round's timeout (non-blocking ncclCommSplit polled on the host): a member that dies
            # between the agreement above and the split turns into a PeerFailure, not a hang
            made = child.split_from(self.rccl, -1 if leaving else 0, 0 if leaving else members.index(rdzv.wid),
                                    timeout_s=self.timeout_s)
        except RuntimeError as exc:
            raise PeerFailure(str(exc)) from exc
        if leaving or not made:
            return "leave", None
        return "split", (members, child)

    def release(self):
        """Drop the RCCL communicator of a round whose successor was built (shrunk from it or not)."""
        if self.rccl is not None:
            self.rccl.abort()
            self.rccl = None

    # -- data plane ------------------------------------------------------------------------------
    def allreduce_async(self, t: torch.Tensor, avg: bool = False):
        if self.rccl is not None and self.emulated:
            return _CpuWork(self.rccl.allreduce_async(t, avg))
        if self.rccl is not None:
            self.rccl.allreduce_(t, 1 if avg else 0)
            ev = torch.cuda.Event()
            ev.record()
            return _GpuWork(self, ev)
        return _CpuWork(dist.all_reduce(t, op=dist.ReduceOp.SUM, async_op=True))

    def broadcast_(self, t: torch.Tensor, src: int):
        if self.rccl is not None and self.emulated:
            try:
                return self.rccl.broadcast_(t, src)
            except RuntimeError as exc:
                raise PeerFailure(str(exc)) from exc
        if self.rccl is not None:
            self.rccl.broadcast_(t, src)
            ev = torch.cuda.Event()
            ev.record()
            self.wait_event(ev)
            return t
        try:
            if t.device.type == "cpu":
                dist.broadcast(t, src)
            else:  # control plane is gloo: stage through the host
                h = t.cpu()
                dist.broadcast(h, src)
                t.copy_(h)
        except RuntimeError as exc:
            raise PeerFailure(str(exc)) from exc
        return t

    def step_done(self, lag: int = 1):
        """Mark the end of a training step.  The host checks the step ``lag`` steps back (its collectives
        finished, or a failure surfaces as :class:`PeerFailure`), so it never stalls on the step it just
        enqueued -- one liveness wait per step instead of one host sync per bucket."""
        if self.rccl is None or self.emulated:
            return
        ev = torch.cuda.Event()
        ev.record()
        self._steps.append(ev)
        while len(self._steps) > lag:
            self.wait_event(self._steps.pop(0))

    def drain(self):
        """Commit point: every enqueued step has finished (or a failure surfaces)."""
        while self._steps:
            self.wait_event(self._steps.pop(0))

    def wait_event(self, ev):
        """Host-side liveness wait for an RCCL collective: returns when it finished; aborts the
        communicator and raises :class:`PeerFailure` on an RCCL async error, when the collective is
        still pending ``grace_s`` after the driver published a newer round, or after ``timeout_s``."""
        t0 = time.time()
        next_check = t0 + 0.05
        while not ev.query():
            now = time.time()
            if now >= next_check:
                next_check = now + 0.05
                err = self.rccl.async_error()
                if err not in (0, 7):  # ncclSuccess, ncclInProgress
                    self.abort()
                    raise PeerFailure(f"RCCL async error {err}")
                if now - t0 > self.grace_s and self.rdzv.hosts_updated():
                    self.abort()
                    raise PeerFailure("collective stalled after a membership change")
                if now - t0 > self.timeout_s:
                    self.abort()
                    raise PeerFailure(f"collective timed out after {self.timeout_s}s")
            time.sleep(0.0002)

    # -- control plane ---------------------------------------------------------------------------
    def agree(self, flag: bool) -> bool:
        t = torch.tensor([1.0 if flag else 0.0])
        try:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        except RuntimeError as exc:
            raise PeerFailure(str(exc)) from exc
        return bool(t.item() > 0)

    def broadcast_object(self, obj, src: int = 0):
        lst = [obj if self.rank == src else None]
        try:
            dist.broadcast_object_list(lst, src=src)
        except RuntimeError as exc:
            raise PeerFailure(str(exc)) from exc
        return lst[0]

    def abort(self):
        if self.rccl is not None:
            self.rccl.abort()

    def close(self, abort: bool = False, keep_rccl: bool = False):
        """End of the round.  ``keep_rccl``: leave the RCCL communicator alive as the next round's shrink
        parent (released by that round); the gloo control group is always torn down."""
        if self.rccl is not None and not abort and not self.emulated:
            try:
                self.drain()
            except PeerFailure:
                abort = True
        self._steps = []
        if self.rccl is not None and keep_rccl:
            pass
        elif self.rccl is not None:
            if abort:
                self.rccl.abort()
            else:
                try:
                    self.rccl.destroy()
                except RuntimeError:
                    self.rccl.abort()
            self.rccl = None
        try:
            if dist.is_initialized():
                dist.destroy_process_group()
        except Exception:  # noqa: BLE001 - a group with a dead member may fail to tear down cleanly
            pass


def _to_cpu(obj):
    if torch.is_tensor(obj):
        return obj.detach().cpu()
    if isinstance(obj, dict):
        return type(obj)((k, _to_cpu(v)) for k, v in obj.items())
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_cpu(v) for v in obj)
    return obj


class Commit:
    """In-memory commit of model + optimizer + position (device-resident clones)."""

    def __init__(self, model, optimizer, position: dict):
        self.model, self.optimizer = model, optimizer
        self.position = position
        self.save()

    def save(self):
        self._model = _clone(self.model.state_dict())
        self._opt = _clone(self.optimizer.state_dict())
        self._pos = dict(self.position)

    def restore(self):
        self.model.load_state_dict(self._model)
        self.optimizer.load_state_dict(_clone(self._opt))
        self.position.clear()
        self.position.update(self._pos)


class _DeviceCommit:
    """Commit points of the fused GPU step without a device synchronisation.

    All trainable state of the fused CNN is ONE flat fp32 tensor (plain SGD keeps no other state).  ``save()``
    enqueues a copy of it into one of two device buffers and records an event, together with the host-side
    position; a pending commit is CONFIRMED once its event has completed and the xGMI exchange's host-mapped
    error word is still clear (a timed-out exchange before the copy would have set it first).  ``throttle()``
    waits for the previous commit's event only: the host stays at most one commit interval ahead of the device, so
    failures surface within an interval while the GPU always has an interval of replays queued.
    ``restore()`` (after a PeerFailure) copies the last confirmed commit back; ``Commit``'s clone of the optimiser
    state dict is kept for the (tiny) step counter."""

    def __init__(self, flat: torch.Tensor, model, optimizer, position: dict, failed=None):
        self.flat, self.position = flat, position
        self.failed = failed or (lambda: False)
        self.bufs = [torch.empty_like(flat), torch.empty_like(flat)]
        self.host = Commit(model, optimizer, position)  # synchronous baseline commit (round start)
        self.bufs[0].copy_(flat)
        torch.cuda.synchronize()
        self.confirmed = (0, dict(position))
        self.pending = None
        self.last_event = None
        self.saves = self.skipped = 0

    def _promote(self, wait: bool = False):
        if self.pending is None:
            return
        slot, ev, pos = self.pending
        if wait:
            ev.synchronize()
        elif not ev.query():
            return
        if not self.failed():
            self.confirmed = (slot, pos)
        self.pending = None

    def throttle(self):
        if self.last_event is not None:
            self.last_event.synchronize()

    def save(self):
        """Non-blocking commit at the current position (no host sync; skipped while the last one is in flight)."""
        self._promote()
        if self.pending is not None:
            self.skipped += 1
            return
        slot = 1 - self.confirmed[0]
        self.bufs[slot].copy_(self.flat)
        ev = torch.cuda.Event()
        ev.record()
        self.pending = (slot, ev, dict(self.position))
        self.last_event = ev
        self.saves += 1

    def save_sync(self):
        """Commit now and wait for it (epoch end: the device is synchronised there anyway)."""
        self._promote(wait=True)
        self.save()
        self._promote(wait=True)

    def restore(self):
        try:
            torch.cuda.synchronize()
        except RuntimeError:
            pass
        self._promote(wait=False)
        self.pending = None
        slot, pos = self.confirmed
        with torch.no_grad():
            self.flat.copy_(self.bufs[slot])
        self.position.clear()
        self.position.update(pos)

    @property
    def _pos(self):  # (the log line of the failure path reads the restored position)
        return self.confirmed[1]


def _as_peer_failure(fn):
    """Run a data-/control-plane call of the round; its RuntimeError (an xGMI exchange that timed out on a dead
    peer, a gloo collective or store wait whose peer vanished) becomes :class:`PeerFailure`, which the re-wire
    loop survives -- never a raw error that would take the survivors down with the dead peer."""
    try:
        return fn()
    except PeerFailure:
        raise
    except RuntimeError as exc:
        raise PeerFailure(str(exc)) from exc


def run_elastic(args):
    """``mnist_ddp_elastic.py --rewire``: the Trainer loop of apps/mnist_ddp.py with in-process re-wire."""
    from ..apps.mnist_ddp import load_train_objs
    from ..data.loader import ShardedLoader
    from ..elastic.snapshot import save_snapshot
    from ..parallel import dist as pdist
    from ..parallel.ddp import DistributedDataParallel
    from ..utils import config as rtconfig
    from ..utils.log import RankLogger

    if "PDE_ELASTIC_STORE" not in os.environ:
        raise SystemExit("--rewire needs the elastic driver: python -m pytorch_distributed_examples_amd.launch.hvdrun "
                         "-np N --min-np M pytorch_elastic/mnist_ddp_elastic.py E S --rewire")
    rdzv = RendezvousClient()
    use_gpu = args.device != "cpu" and torch.cuda.is_available()
    if use_gpu:
        local = int(os.environ.get("LOCAL_RANK", "0"))
        dev = torch.device("cuda", local % torch.cuda.device_count())
        torch.cuda.set_device(dev)
    else:
        dev = torch.device("cpu")
    train_set, test_set, model, make_opt, criterion = load_train_objs(args.model, dev, args.train_size,
                                                                      args.test_size)
    model = model.to(dev)
    optimizer = make_opt(model.parameters())
    pos = {"epoch": 0, "seen": 0}  # samples of the current epoch consumed by the whole group
    commit = Commit(model, optimizer, pos)
    commit_every = max(1, int(getattr(args, "commit_every", 10)))
    step = 0
    ddp = None
    pid = os.getpid()
    parent = None  # previous round's communicator set, kept as a possible shrink parent
    premade = None  # (members, communicator) split off the previous round for a planned scale-down
    while True:
        rnd, rank, size = rdzv.join()
        comm = RoundComm(rdzv, rank, size, dev, parent=parent, premade=premade)
        parent = premade = None
        log = RankLogger(rank)
        log.print(f"[rewire] round {rnd}: rank {rank} of {size} (pid {pid}, rccl {comm.how})", all_ranks=True)
        try:
            # rank 0 is a survivor with the newest commit: everybody adopts its state
            state = comm.broadcast_object({"pos": dict(pos), "opt": _to_cpu(optimizer.state_dict())}
                                          if rank == 0 else None)
            if rank != 0:
                pos.clear()
                pos.update(state["pos"])
                optimizer.load_state_dict(state["opt"])
            if ddp is not None:
                ddp.remove_hooks()
            ddp = DistributedDataParallel(model, comm=comm, **rtconfig.from_args(args).ddp_kwargs())
            commit.save()
            train_data = ShardedLoader(train_set, args.batch_size, size, rank, shuffle=True)
            test_data = ShardedLoader(test_set, args.batch_size, size, rank, shuffle=False)
            per_step = args.batch_size * size
            since = 0
            for epoch in range(pos["epoch"], args.total_epochs):
                model.train()
                train_data.set_epoch(epoch)
                train_data.start_batch = min(pos["seen"] // per_step, len(train_data))
                log.print(f"Local Rank: {rdzv.wid} | Global Rank: {rank} | Epoch {epoch} | Batchsize: "
                          f"{args.batch_size} | Steps: {len(train_data)} | start batch {train_data.start_batch}",
                          all_ranks=True)
                for source, targets in train_data:
                    ddp.zero_grad()
                    loss = criterion(ddp(source), targets)
                    loss.backward()
                    optimizer.step()
                    comm.step_done()
                    fault.maybe_fault(step, rank)
                    step += 1
                    pos["seen"] += per_step
                    since += 1
                    if since % commit_every == 0:
                        comm.drain()
                        commit.save()
                        if comm.agree(rdzv.hosts_updated()):
                            raise MembershipChanged()
                pos["epoch"], pos["seen"] = epoch + 1, 0
                comm.drain()
                commit.save()
                _test(model, test_data, dev, comm, log)
                if rank == 0 and epoch % args.save_every == 0:
                    save_snapshot(args.snapshot_path, model.state_dict(), epoch, optimizer.state_dict())
                    log.print(f"Epoch {epoch} | Training snapshot saved at {args.snapshot_path}")
            log.print(f"[rewire] finished {args.total_epochs} epochs in round {rnd} (world {size}, pid {pid})",
                      all_ranks=True)
            comm.close()
            break
        except PeerFailure as exc:
            log.print(f"[rewire] round {rnd}: peer failure ({str(exc).splitlines()[0][:120]}); restoring commit "
                      f"epoch {commit._pos['epoch']} seen {commit._pos['seen']}", all_ranks=True)
            # a communicator the failure already aborted cannot be a shrink parent (RoundComm re-checks
            # validity on every survivor and agrees before anyone calls ncclCommShrink)
            keep = comm.rccl is not None and comm.rccl.valid and comm.rccl.shrink_supported()
            comm.close(abort=not keep, keep_rccl=keep)  # a shrink (ABORT flag) tears its work down
            parent = comm if keep else None
            commit.restore()
        except MembershipChanged:
            log.print(f"[rewire] round {rnd}: membership changed, re-joining", all_ranks=True)
            try:  # every member is alive here: a scale-down splits the communicator instead of re-initialising
                how, premade = comm.planned_split()
            except PeerFailure:
                how, premade = "none", None
            comm.close()
            if how == "leave":
                log.print(f"[rewire] round {rnd}: leaving the job (planned scale-down, pid {pid})", all_ranks=True)
                break
    pdist.shutdown()


@torch.no_grad()
def _test(model, loader, dev, comm, log):
    was = model.training
    model.eval()
    correct = torch.zeros((), dtype=torch.long, device=dev)
    total = 0
    for images, labels in loader:
        correct += (model(images).float().argmax(1) == labels).sum()
        total += labels.size(0)
    t = torch.tensor([float(correct.item()), float(total)])
    if comm.size > 1:
        try:
            dist.all_reduce(t)
        except RuntimeError as exc:
            raise PeerFailure(str(exc)) from exc
    log.print(f"Global test accuracy: {t[0].item() / max(1.0, t[1].item()) * 100:.2f}%")
    model.train(was)


class _FailureWatch:
    """Background watcher of one round: when the elastic driver reports a failed member of THIS round
    (``failed/<round>`` in its store, set the moment it reaps the dead process) it raises the xGMI exchange's
    host abort word, so the survivors' spinning in-kernel exchanges give up within ~0.1 ms instead of waiting
    out their timeout (detection used to cost the 5 s timeout plus a commit interval).
    A planned membership change (hosts added / removed by discovery) publishes no failure: it is handled at the
    next commit point without dropping any step."""

    def __init__(self, rdzv: RendezvousClient, rnd: int, xa, period_s: float = 0.02):
        import threading

        self.rnd, self.xa, self.period_s = rnd, xa, period_s
        self.fired_at = None
        self._stop = threading.Event()
        addr = os.environ["PDE_ELASTIC_STORE"]
        # a client of its own (never interleaves with the main thread's store traffic), reused by the next round's
        # watcher once this one has stopped: one connection per process, not one per elastic reset
        self._store = _WATCH_STORES.pop(addr, None)
        if self._store is None:
            host, port = addr.rsplit(":", 1)
            self._store = dist.TCPStore(host, int(port), is_master=False, timeout=datetime.timedelta(seconds=30),
                                        wait_for_workers=False)
        self._addr = addr
        self._th = threading.Thread(target=self._run, daemon=True)
        self._th.start()

    def _run(self):
        key = f"failed/{self.rnd}"
        while not self._stop.wait(self.period_s):
            try:
                if self._store.check([key]):
                    self.fired_at = time.time()
                    if self.xa is not None and self.xa.impl is not None:
                        self.xa.abort()
                    return
            except Exception:  # noqa: BLE001 - the driver went away: the main thread sees it too
                return

    def stop(self):
        self._stop.set()
        self._th.join(timeout=1.0)
        store, self._store = self._store, None
        if store is not None and not self._th.is_alive():
            _WATCH_STORES[self._addr] = store  # idle again: hand it to the next round's watcher
        # else the thread is still inside a store call: drop our reference, it is released when the call returns


_WATCH_STORES: dict = {}  # PDE_ELASTIC_STORE address -> an idle watcher TCPStore client


def _fault_time():
    """Wall-clock time the injected fault fired (PDE_FAULT_ONCE marker, elastic/fault.py), if any."""
    marker = os.environ.get("PDE_FAULT_ONCE")
    if not marker or not os.path.exists(marker):
        return None
    try:
        for tok in open(marker).read().split():
            if tok.startswith("t="):
                return float(tok[2:])
    except (OSError, ValueError):
        return None
    return None


def run_elastic_fused(args, report=None):
    """``mnist_ddp_elastic.py --rewire --model cnn --fused`` and the elastic bench (BASELINE config 2).

    The reference trainer's semantics (pytorch_elastic/mnist_ddp_elastic.py:82-114) on the fused path:
    epochs over this rank's ``DistributedSampler`` shard of the training set (:class:`..data.loader.ShardedLoader`,
    re-sharded for the new world after every membership change and resumed at the first batch the whole group
    has not consumed, ``pos["seen"]``), a test pass over the sharded test set after every epoch (accuracy
    all-reduced), and rank 0's snapshot every ``save_every`` epochs with the reference's keys.

    The step is the fused whole-network CNN with the gradient exchange over xGMI INSIDE its reduction kernel
    (``FusedCNN.forward_backward(..., xgmi=...)``: 2 launches per step at any world size) and the SGD update fused
    in.  ``graph_steps`` steps are recorded into ONE hipGraph per round whose inputs are ``graph_steps`` static
    batch slots, preceded by ONE gather node (``gather_rows_counter``) that copies the next ``graph_steps`` batches
    of the epoch's shard into the slots, at the position of a DEVICE replay counter it advances itself -- every
    replay trains on new data with no host work between replays (the host writes the counter once per epoch /
    resume).  The first step of a round, a resumed position inside a replay and an epoch's tail run as eager fused
    steps.  The graph is recaptured after every membership change (xGMI view and world size are baked in).

    Commit points (every ``commit_every`` replays) never synchronise the device (:class:`_DeviceCommit`): the
    weights are copied on the stream into one of two device buffers behind an event, and a commit is CONFIRMED
    once its event has completed with the exchange's host-mapped error word still clear; the host waits only for
    the PREVIOUS commit's event, so at most one interval of replays is queued and the GPU never idles.  Liveness:
    the failure watch's abort word (the driver reports a dead member) or the error word turns into PeerFailure at
    the next commit point, and the survivors restore the last confirmed commit.

    Failure handling: a dead peer makes the exchange give up -- at once when the driver reports the failure
    (:class:`_FailureWatch` raises the exchange's host abort word), else at its timeout -- and the next commit
    point (every ``commit_every`` replays: ``xgmi.check()`` + the gloo ``agree``) turns it into PeerFailure:
    the survivors restore their last commit and re-join in-process.  ``detect_s`` (the fault -> PeerFailure
    latency, from the injector's timestamp) is reported with the re-wire breakdown.

    ``report(round, rank, size, info)`` (bench): called by every rank after each round's timed window (whole
    replays inside one epoch, so no test pass or epoch tail falls inside it) with img/s and the re-wire latency
    (membership change seen -> first step of the new round complete); returning True ends training."""
    import time as _time

    from ..data.loader import ShardedLoader
    from ..data.synthetic import mnist_splits
    from ..elastic.snapshot import save_snapshot
    from ..models.cnn import Net
    from ..models.cnn_fused import FusedCNN
    from ..ops.optim import FusedSGD
    from ..parallel import dist as pdist
    from ..parallel.xgmi_allreduce import XgmiAllreduce
    from ..utils.epoch_graph import sampler_indices
    from ..utils.graph import CapturedSteps
    from ..utils.log import RankLogger

    if "PDE_ELASTIC_STORE" not in os.environ:
        raise SystemExit("--rewire needs the elastic driver (launch.hvdrun)")
    rdzv = RendezvousClient()
    local = int(os.environ.get("LOCAL_RANK", "0"))
    on_gpu = torch.cuda.is_available() and getattr(args, "device", "auto") != "cpu"
    if on_gpu:
        dev = torch.device("cuda", local % torch.cuda.device_count())
        torch.cuda.set_device(dev)
    else:  # CPU plumbing of the same protocol: autograd Net + DDP over the round's gloo group, eager steps
        dev = torch.device("cpu")
        torch.set_num_threads(1)
    torch.manual_seed(0)
    model = Net().to(dev).train()
    fused = FusedCNN(model) if on_gpu else None
    grads = fused.grad_buffer() if on_gpu else None
    opt = FusedSGD(model.parameters(), lr=0.01)

    def sync():
        if on_gpu:
            torch.cuda.synchronize()

    batch = int(args.batch_size)
    G = max(1, int(getattr(args, "graph_steps", 10)))
    # the reference's MNIST sizes (synthetic, HBM-resident); a bench may ask for a longer VIRTUAL epoch
    # (indices wrap around the real samples) so its timed window never straddles an epoch boundary
    real_train = int(getattr(args, "train_size", 60000))
    virt_train = int(getattr(args, "virtual_train_size", 0) or real_train)
    train_set, test_set = mnist_splits(device=dev, train=real_train, test=int(getattr(args, "test_size", 10000)))
    train_view = train_set
    if virt_train != real_train:
        class _Virtual:  # a longer epoch over the same samples (ShardedLoader only needs len())
            def __len__(self):
                return virt_train
        train_view = _Virtual()
    total_epochs = int(getattr(args, "total_epochs", 1))
    total_steps = int(getattr(args, "total_steps", 0) or 0)  # > 0: stop after this many steps (bench)
    save_every = int(getattr(args, "save_every", 0) or 0)
    snapshot_path = getattr(args, "snapshot_path", None)
    # static batch slots of the captured group (GPU): replay j trains on slot j
    xbuf = torch.empty(G * batch, 1, 28, 28, device=dev)
    ybuf = torch.zeros(G * batch, dtype=torch.long, device=dev)
    slots = [(xbuf[j * batch:(j + 1) * batch], ybuf[j * batch:(j + 1) * batch]) for j in range(G)]
    # the graph's gather reads the epoch's index list at a fixed address and the replay position from a device
    # counter (int32 [replay, done-count]), written by the host once per epoch / resume
    counter = torch.zeros(2, dtype=torch.int32, device=dev) if on_gpu else None
    pos = {"epoch": 0, "seen": 0, "step": 0}
    commit = Commit(model, opt, pos)
    commit_every = max(1, int(getattr(args, "commit_every", 10)))  # graph replays between commit points
    changed_at = None
    detect = None
    pid = os.getpid()

    def gather(idx, lo, hi, xo, yo):
        sl = idx[lo:hi]  # (already reduced modulo the real sample count)
        torch.index_select(train_set.images, 0, sl, out=xo)
        torch.index_select(train_set.labels, 0, sl, out=yo)

    while True:
        t_join = _time.perf_counter()
        rnd, rank, size = rdzv.join()
        t_joined = _time.perf_counter()
        comm = RoundComm(rdzv, rank, size, dev, use_rccl=False)
        log = RankLogger(rank)
        xa = None
        watch = None
        dcommit = None
        parts = {"rendezvous_s": t_joined - (changed_at if changed_at is not None else t_join),
                 "control_s": comm.timing.get("control_group_s", 0.0)}
        try:
            tb = _time.perf_counter()
            if size > 1:  # everybody adopts rank 0's weights and position (87 KB over the control plane)
                if on_gpu:
                    comm.broadcast_(fused.flat, 0)
                else:
                    for p_ in model.parameters():
                        comm.broadcast_(p_.data, 0)
            state = comm.broadcast_object(dict(pos) if rank == 0 else None) if size > 1 else dict(pos)
            pos.clear()
            pos.update(state)
            round_step0 = pos["step"]  # the round's first step runs eagerly (then the graph is captured)
            sync()
            parts["broadcast_s"] = _time.perf_counter() - tb
            tm = _time.perf_counter()
            if on_gpu:
                fused.invalidate()
                xa = _as_peer_failure(lambda: XgmiAllreduce(dev, key=f"rewire/{rnd}")) if size > 1 else None
                parts["map_s"] = _time.perf_counter() - tm
                tc = _time.perf_counter()

                def train_step(x, y):
                    return fused.forward_backward(x, y, grad_out=grads, sgd=opt, xgmi=xa)

                graph = None  # captured at the round's first replay point, after one eager step
                eager_step = train_step
                C_ = _native.C()
                idx_buf = None
            else:
                from ..ops import functional as OF
                from ..parallel.ddp import DistributedDataParallel

                ddp = DistributedDataParallel(model, comm=comm, overlap=False)
                parts["map_s"] = _time.perf_counter() - tm
                tc = _time.perf_counter()

                def eager_step(x, y):
                    ddp.zero_grad()
                    out = OF.nll_loss(model(x), y)
                    out.backward()
                    ddp.sync_gradients()
                    opt.step()
                    return out

                class _Eager:  # CapturedSteps' replay() surface over eager steps on the slots
                    def replay(self):
                        out = None
                        for x, y in slots:
                            out = eager_step(x, y)
                        return out

                graph = _Eager()
            sync()
            parts["capture_s"] = _time.perf_counter() - tc
            if detect is not None:
                parts["detect_s"] = detect
            rewire_s = _time.perf_counter() - changed_at if changed_at is not None else None
            changed_at = detect = None
            watch = _FailureWatch(rdzv, rnd, xa) if size > 1 else None
            if on_gpu:
                dcommit = _DeviceCommit(fused.flat, model, opt, pos,
                                        failed=(lambda: xa.failed()) if xa is not None else None)
            plane = f"fused CNN + xGMI exchange, {G} steps per graph" if on_gpu else "CPU autograd + gloo DDP"
            log.print(f"[rewire] round {rnd}: rank {rank} of {size} (pid {pid}), {plane}" +
                      (f", re-wired in {rewire_s:.3f}s (" + ", ".join(f"{k[:-2]} {v:.3f}" for k, v in parts.items())
                       + ")" if rewire_s is not None else ""), all_ranks=True)
            if not on_gpu:
                commit.save()
            train_data = ShardedLoader(train_view, batch, size, rank, shuffle=True)
            test_data = ShardedLoader(test_set, batch, size, rank, shuffle=False)
            per_step = batch * size
            n_batches = len(train_data)
            window = None
            if report is not None:  # the bench's timed window: warm-up + timed replays at an epoch start
                window = {"warm": int(getattr(args, "round_warmup", 2)), "timed": int(getattr(args, "round_replays", 10)),
                          "done": False}
                if (window["warm"] + window["timed"]) * G > n_batches:
                    raise SystemExit(f"elastic bench: the timed window needs {(window['warm'] + window['timed']) * G} "
                                     f"batches per epoch, the shard has {n_batches}: raise virtual_train_size")
            since = 0
            stop = False
            while not stop:
                epoch = pos["epoch"]
                if total_steps:
                    if pos["step"] >= total_steps:
                        break
                elif epoch >= total_epochs:
                    break
                train_data.set_epoch(epoch)
                idx = sampler_indices(train_data.sampler) % real_train
                if on_gpu:  # the graph's gather reads this buffer: same address every epoch of the round
                    if idx_buf is None or idx_buf.numel() != idx.numel():
                        idx_buf, graph = torch.empty(idx.numel(), dtype=torch.long, device=dev), None
                    idx_buf.copy_(idx)
                    idx = idx_buf
                b = min(pos["seen"] // per_step, n_batches)  # resume after the group's consumed batches
                at = None  # the replay index the device counter holds (None: unknown -> rewritten before a replay)
                log.print(f"Local Rank: {rdzv.wid} | Global Rank: {rank} | Epoch {epoch} | Batchsize: {batch} | "
                          f"Steps: {n_batches} | start batch {b}", all_ranks=True)
                # the bench window: whole replays inside this epoch (no test pass or eager tail inside it); a round
                # resuming too close to the epoch's end times the next epoch
                timing = window is not None and not window["done"] and \
                    n_batches - b >= (window["warm"] + window["timed"]) * G
                replays = 0
                t0 = None
                loss = None
                while b < n_batches:
                    if total_steps and pos["step"] >= total_steps:
                        stop = True
                        break
                    step0 = pos["step"]
                    if on_gpu and b % G == 0 and b + G <= n_batches and (b + G) * batch <= idx.numel() and \
                            (graph is not None or pos["step"] > round_step0):
                        if graph is None:  # after >= 1 eager step of this round initialised everything
                            def gather_slots():
                                C_.gather_rows_counter(train_set.images, train_set.labels, idx_buf, counter, xbuf,
                                                       ybuf)
                            graph = CapturedSteps(train_step, slots, warmup=0, prologue=gather_slots).capture()
                        if at != b // G:
                            counter.copy_(torch.tensor([b // G, 0], dtype=torch.int32))
                        loss = graph.replay()  # gather the next G batches at the counter + G fused steps
                        at = b // G + 1
                        n = G
                        replays += 1
                    elif not on_gpu and b + G <= n_batches and (b + G) * batch <= idx.numel():
                        gather(idx, b * batch, (b + G) * batch, xbuf, ybuf)  # the next G batches -> the slots
                        loss = graph.replay()
                        n = G
                        replays += 1
                    else:  # round start, resumed mid-replay, epoch tail: eager fused steps
                        lo, hi = b * batch, min((b + 1) * batch, idx.numel())
                        x, y = xbuf[:hi - lo], ybuf[:hi - lo]
                        gather(idx, lo, hi, x, y)
                        loss = eager_step(x.contiguous(), y.contiguous())
                        n = 1
                    b += n
                    pos["seen"] = b * per_step
                    pos["step"] += n
                    fault.maybe_fault_in(step0, step0 + n, rank)  # PDE_FAULT_*: a step of this replay
                    if timing:
                        if replays == window["warm"] and t0 is None:
                            sync()
                            comm.agree(False)  # barrier over the control plane
                            t0 = _time.perf_counter()
                        elif t0 is not None and replays == window["warm"] + window["timed"]:
                            sync()
                            dt = _time.perf_counter() - t0
                            if xa is not None:
                                _as_peer_failure(xa.check)
                            t = torch.tensor([dt] + [rewire_s if rewire_s is not None else -1.0] + list(parts.values()))
                            if size > 1:  # the slowest member's window and re-wire (one MAX over the control plane)
                                _as_peer_failure(lambda: dist.all_reduce(t, op=dist.ReduceOp.MAX))
                            info = {"images_per_s": per_step * G * window["timed"] / float(t[0].item()),
                                    "ms_per_step": float(t[0].item()) / (G * window["timed"]) * 1e3,
                                    "rewire_s": float(t[1].item()) if t[1].item() >= 0 else None,
                                    "loss": float(loss.item())}
                            if t[1].item() >= 0:
                                info["rewire_parts"] = {k: round(float(v), 4) for k, v in zip(parts, t[2:].tolist())}
                            window["done"] = True
                            timing = False
                            stop = bool(report(rnd, rank, size, info))
                            if stop:
                                break
                    since += 1
                    if since % commit_every == 0:  # commit point: liveness + membership
                        if on_gpu:  # no device sync: bounded queue, non-blocking failure words, device copy
                            dcommit.throttle()
                            if (watch is not None and watch.fired_at is not None) or (xa is not None and xa.failed()):
                                raise PeerFailure("xGMI exchange gave up on a peer (driver-reported failure / "
                                                  "timeout)")
                            dcommit.save()
                        else:
                            sync()
                            commit.save()
                        if comm.agree(rdzv.hosts_updated()):
                            raise MembershipChanged()
                if stop:
                    break
                # end of epoch (mnist_ddp_elastic.py:111-114): commit, test pass, snapshot
                sync()
                if xa is not None:
                    _as_peer_failure(xa.check)
                pos["epoch"], pos["seen"] = epoch + 1, 0
                if on_gpu:
                    dcommit.save_sync()
                else:
                    commit.save()
                _test(model, test_data, dev, comm, log)
                if rank == 0 and save_every and snapshot_path and epoch % save_every == 0:
                    save_snapshot(snapshot_path, model.state_dict(), epoch, opt.state_dict())
                    log.print(f"Epoch {epoch} | Training snapshot saved at {snapshot_path}")
                if comm.agree(rdzv.hosts_updated()):
                    raise MembershipChanged()
            log.print(f"[rewire] finished {pos['step']} steps / {pos['epoch']} epochs in round {rnd} (world {size}, "
                      f"pid {pid})", all_ranks=True)
            if watch is not None:
                watch.stop()
            if xa is not None:
                xa.close()
            comm.close()
            break
        except PeerFailure as exc:
            changed_at = _time.perf_counter()
            tf = _fault_time()
            detect = (time.time() - tf) if tf is not None else None
            log.print(f"[rewire] round {rnd}: peer failure ({str(exc).splitlines()[0][:120]}); restoring commit "
                      f"epoch {(dcommit or commit)._pos['epoch']} step {(dcommit or commit)._pos['step']}" +
                      (f"; detected {detect:.3f}s after the fault" if detect is not None else ""), all_ranks=True)
            comm.close(abort=True)
            if on_gpu and dcommit is not None:
                dcommit.restore()
            else:
                commit.restore()
            if fused is not None:
                fused.invalidate()
        except MembershipChanged:
            changed_at = _time.perf_counter()
            log.print(f"[rewire] round {rnd}: membership changed, re-joining", all_ranks=True)
            comm.close()
        finally:
            if watch is not None:
                watch.stop()
            if xa is not None and xa.impl is not None:
                torch.cuda.synchronize()
                xa.close()
    pdist.shutdown()
