"""``RemoteModule``: a module hosted by another process (rpc/server_model_data_parallel.py:134-139).

``RemoteModule("ps", nn.EmbeddingBag, args=(100, 16), kwargs={"mode": "sum"})`` builds the module on
worker "ps" (on its GPU when it has one: the EmbeddingBag gather / scatter-add are HIP kernels) and
returns a picklable handle; ``forward(*args)`` is a synchronous RPC whose result is attached to the
caller's autograd graph, and whose backward ships the output gradient back to the owner, which
accumulates it per distributed-autograd context.

GPU data plane (``forward(..., out_device=cuda)`` with the module on a GPU): the RPC carries only the
call and the (small, host) indices / offsets; the looked-up rows go owner GPU -> caller GPU through a
P2P receive ring over xGMI (csrc/comm/p2p_ring.hip, one ring pair per caller, IPC handles exchanged by RPC
on first use), and the output gradient goes back the same way -- no ``.cpu()`` on the lookup or the
gradient path (the reference's dist autograd moves both as CPU tensors, server_model_data_parallel.py:45,
102).  Stream-ordered on both sides: the owner enqueues its send behind the lookup kernel before the RPC
returns, the caller's receive kernel waits for the ring's flags.  ``remote_parameters()`` returns parameter handles for
:class:`~.core.DistributedOptimizer`; each trainer's optimizer updates the owner's table independently
(Hogwild-style, quirk Q16 kept).  Concurrent callers are served in arrival order by the owner's
executor thread.
"""
from __future__ import annotations

import threading

import torch
import torch.distributed.rpc as rpc

from . import core


def _make_server(module_cls, args, kwargs, device):
    return core.ModuleServer(module_cls, args, kwargs, device)


# ---- GPU data plane: one P2P ring pair per (caller process, server) --------------------------------
def _ring_slot_bytes() -> int:
    import os

    return int(float(os.environ.get("PDE_P2P_SLOT_MB", "4")) * (1 << 20))


def _ring_ordered_submit(srv, caller: str, idx: int, fn) -> torch.futures.Future:
    """Run ``fn`` on the owner's executor in ring-message order for ``caller``: ``idx`` is the caller's index
    of the ring message ``fn`` receives.  The caller sends its gradient messages in autograd order but their
    RPCs may be delivered out of order by the agent's thread pool (several remote calls per context), and a
    receive must take the message that belongs to its call -- so receives are queued by index, not arrival."""
    out = torch.futures.Future()
    lock = srv.__dict__.setdefault("_ring_lock", threading.Lock())
    with lock:
        st = srv.__dict__.setdefault("_ring_order", {}).setdefault(caller, {"next": 0, "pending": {}})
        st["pending"][idx] = (fn, out)
        while st["next"] in st["pending"]:
            f, fut = st["pending"].pop(st["next"])
            st["next"] += 1

            def _relay(done, fut=fut):
                try:
                    fut.set_result(done.value())
                except Exception as exc:  # noqa: BLE001 - the RPC caller sees the owner's error
                    fut.set_exception(exc)

            srv.submit(f).add_done_callback(_relay)  # FIFO executor: submission order is execution order
    return out


def _rm_open_ring(srv_rref, caller: str, caller_handle: bytes):
    """Owner side of the ring handshake: a ring for ``caller``, mapped to the caller's; returns its handle."""
    from .. import _native

    srv = srv_rref.local_value()

    def run():
        rings = srv.__dict__.setdefault("rings", {})
        ring = _native.comm().P2PRing(srv.device.index, _ring_slot_bytes(), 60.0)
        ring.open(caller_handle)
        rings[caller] = ring
        srv.__dict__.setdefault("_ring_order", {}).pop(caller, None)  # a new ring restarts the message index
        return ring.ipc_handle()

    return srv.submit(run).wait()


def _rm_close_ring(srv_rref, caller: str):
    srv = srv_rref.local_value()

    def run():
        ring = getattr(srv, "rings", {}).pop(caller, None)
        if ring is not None:
            ring.close()
        return True

    return srv.submit(run).wait()


@rpc.functions.async_execution
def _rm_forward_ring(srv_rref, ctx_id, call_id, caller, args):
    srv = srv_rref.local_value()

    def run():
        dev_args = [a.to(srv.device) if torch.is_tensor(a) else a for a in args]
        out = srv.module(*dev_args)
        srv.saved[(ctx_id, call_id)] = (None, out)
        o = out.detach()
        if o.dtype != torch.float32:
            o = o.float()
        srv.rings[caller].send(o.contiguous())  # owner GPU -> caller GPU, behind the lookup kernel
        return tuple(o.shape)

    return srv.submit(run)


@rpc.functions.async_execution
def _rm_backward_ring(srv_rref, ctx_id, call_id, caller, shape, ring_idx):
    srv = srv_rref.local_value()

    def run():
        _, out = srv.saved.pop((ctx_id, call_id))
        g = torch.empty(shape, dtype=torch.float32, device=srv.device)
        srv.rings[caller].recv(g)  # caller GPU -> owner GPU: message ring_idx of this caller
        torch.autograd.backward(out, g.to(out.dtype))
        core.accumulate_grads(srv, ctx_id)
        return True

    return _ring_ordered_submit(srv, caller, ring_idx, run)


@rpc.functions.async_execution
def _rm_forward(srv_rref, ctx_id, call_id, args):
    srv = srv_rref.local_value()

    def run():
        dev_args = [a.to(srv.device) if torch.is_tensor(a) else a for a in args]
        out = srv.module(*dev_args)
        srv.saved[(ctx_id, call_id)] = (None, out)
        return out.detach().float().cpu()

    return srv.submit(run)


@rpc.functions.async_execution
def _rm_backward(srv_rref, ctx_id, call_id, grad):
    srv = srv_rref.local_value()

    def run():
        _, out = srv.saved.pop((ctx_id, call_id))
        torch.autograd.backward(out, grad.to(srv.device).to(out.dtype))
        core.accumulate_grads(srv, ctx_id)
        return True

    return srv.submit(run)


class RemoteModule:
    def __init__(self, remote_device: str, module_cls, args=(), kwargs=None):
        if "/" in remote_device:
            worker, device = remote_device.split("/", 1)
        else:
            worker, device = remote_device, "cpu"
        self.worker = worker
        self.device = device
        self.server = rpc.remote(worker, _make_server, args=(module_cls, tuple(args), kwargs or {}, device))
        self.server._get_future().wait()  # wait for construction; the server stays on its owner

    # -- GPU data plane ---------------------------------------------------------------------------
    def _ring(self, device: torch.device):
        """This process's ring towards the owner (created + handshaken by RPC on first use)."""
        from .. import _native

        ring = self.__dict__.get("_p2p")
        if ring is None:
            ring = _native.comm().P2PRing(device.index, _ring_slot_bytes(), 60.0)
            me = rpc.get_worker_info().name
            ring.open(rpc.rpc_sync(self.worker, _rm_open_ring, args=(self.server, me, ring.ipc_handle())))
            self.__dict__["_p2p"] = ring
            self.__dict__["_p2p_sent"] = 0  # index of the next message this process sends on the ring
        return ring

    def close(self):
        """Tear down this process's ring towards the owner (and the owner's side); both drain first."""
        ring = self.__dict__.pop("_p2p", None)
        self.__dict__.pop("_p2p_sent", None)
        if ring is not None:
            torch.cuda.synchronize()
            rpc.rpc_sync(self.worker, _rm_close_ring, args=(self.server, rpc.get_worker_info().name))
            ring.close()

    def __getstate__(self):  # the handle travels to other processes; a ring is per process
        d = dict(self.__dict__)
        d.pop("_p2p", None)
        d.pop("_p2p_sent", None)
        return d

    def uses_ring(self, out_device) -> bool:
        return (out_device is not None and torch.device(out_device).type == "cuda"
                and self.device.startswith("cuda"))

    def forward(self, *args, out_device=None):
        """Remote call; ``out_device`` (a GPU of this process, the module on a GPU): the result arrives there
        over the P2P ring instead of as a CPU tensor."""
        ctx = core.current_context()
        call = next(ctx.calls)
        if self.uses_ring(out_device):
            dev = torch.device(out_device)
            ring = self._ring(dev)
            me = rpc.get_worker_info().name
            host_args = tuple(a.cpu() if torch.is_tensor(a) and a.is_cuda else a for a in args)
            shape = rpc.rpc_sync(self.worker, _rm_forward_ring, args=(self.server, ctx.id, call, me, host_args))
            out = torch.empty(shape, dtype=torch.float32, device=dev)
            ring.recv(out)
            return core.attach(out, self.server, ctx, call, self._backward_ring)
        out = rpc.rpc_sync(self.worker, _rm_forward, args=(self.server, ctx.id, call, args))
        return core.attach(out, self.server, ctx, call, self._backward)

    def _backward_ring(self, owner, ctx_id, call_id, grad):
        g = grad.float().contiguous()
        ring = self._ring(g.device)
        idx = self.__dict__["_p2p_sent"]
        self.__dict__["_p2p_sent"] = idx + 1
        ring.send(g)
        me = rpc.get_worker_info().name
        return rpc.rpc_async(self.worker, _rm_backward_ring,
                             args=(self.server, ctx_id, call_id, me, tuple(g.shape), idx))

    __call__ = forward

    def forward_async(self, *args):
        ctx = core.current_context()
        call = next(ctx.calls)
        fut = rpc.rpc_async(self.worker, _rm_forward, args=(self.server, ctx.id, call, args))
        return fut.then(lambda f: core.attach(f.wait(), self.server, ctx, call, self._backward))

    def _backward(self, owner, ctx_id, call_id, grad):
        return rpc.rpc_async(self.worker, _rm_backward, args=(self.server, ctx_id, call_id, grad))

    def remote_parameters(self):
        return core.parameter_rrefs(self.server)
