"""``RemoteModule``: a module hosted by another process (rpc/server_model_data_parallel.py:134-139).

``RemoteModule("ps", nn.EmbeddingBag, args=(100, 16), kwargs={"mode": "sum"})`` builds the module on
worker "ps" (on its GPU when it has one: the EmbeddingBag gather / scatter-add are HIP kernels) and
returns a picklable handle; ``forward(*args)`` is a synchronous RPC whose result is attached to the
caller's autograd graph, and whose backward ships the output gradient back to the owner, which
accumulates it per distributed-autograd context.  ``remote_parameters()`` returns parameter handles for
:class:`~.core.DistributedOptimizer`; each trainer's optimizer updates the owner's table independently
(Hogwild-style, quirk Q16 kept).  Concurrent callers are served in arrival order by the owner's
executor thread.
"""
from __future__ import annotations

import torch
import torch.distributed.rpc as rpc

from . import core


def _make_server(module_cls, args, kwargs, device):
    return core.ModuleServer(module_cls, args, kwargs, device)


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
        self.server = rpc.remote(worker, _make_server, args=(module_cls, tuple(args), kwargs or {}, device))
        self.server._get_future().wait()  # wait for construction; the server stays on its owner

    def forward(self, *args):
        ctx = core.current_context()
        call = next(ctx.calls)
        out = rpc.rpc_sync(self.worker, _rm_forward, args=(self.server, ctx.id, call, args))
        return core.attach(out, self.server, ctx, call, self._backward)

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
