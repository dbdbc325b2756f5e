"""RPC-style remote modules with a device data plane.

The reference drives its model-parallel and parameter-server examples with ``torch.distributed.rpc``
(rpc/model_parallel_ResNet50.py, rpc/server_model_data_parallel.py): remote module construction
(``rpc.remote``/``RemoteModule``), ``RRef``s, async remote calls, distributed autograd and a distributed
optimizer.  This module keeps that programming model but splits it MI355X-first:

* control plane: ``torch.distributed.rpc`` (TensorPipe, CPU) carries only small messages -- calls,
  micro-batch ids, the tiny network outputs / their gradients;
* data plane: stage-to-stage activations and activation-gradients go GPU->GPU over RCCL P2P
  (:class:`..parallel.pipeline.P2PChannel`), never through the RPC agent (ROCm's TensorPipe has no GPU
  channel: SURVEY.md B3);
* each remote module is served by a :class:`ModuleServer` with ONE ordered executor thread (replaces the
  reference's per-shard ``threading.Lock`` + 16-thread pool, :48,:112,:137): calls run in arrival order,
  so RCCL send/recv pairs between stages match without extra synchronisation;
* distributed autograd: a remote call's output is connected to the caller's autograd graph by
  :class:`_RemoteCallFn`; its backward ships the output gradient to the owner asynchronously and the
  owner runs the local backward (and forwards activation gradients upstream over RCCL).
  :func:`dist_autograd_backward` = local ``backward`` + wait for every remote backward of the context.
* :class:`DistributedOptimizer` creates one fused optimizer per parameter owner and steps them by RPC;
  gradients are per-context (``step(context_id)``) like the reference's.
"""
from __future__ import annotations

import contextlib
import itertools
import queue
import threading

import torch
import torch.distributed.rpc as rpc

# --------------------------------------------------------------------------------------------------
# server side
# --------------------------------------------------------------------------------------------------
_SERVERS: dict[int, "ModuleServer"] = {}
_SERVER_IDS = itertools.count(1)


class ModuleServer:
    """Owns a module on this process's device and executes calls in order on one thread."""

    def __init__(self, module_fn, args=(), kwargs=None, device: str = "cpu", setup_fn=None):
        self.device = torch.device(device)
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        self.module = module_fn(*args, **(kwargs or {})).to(self.device)
        self.sid = next(_SERVER_IDS)
        _SERVERS[self.sid] = self
        self.saved: dict = {}  # (ctx, call) -> (inputs, outputs)
        self.grads: dict = {}  # ctx -> {param: grad}
        self.optimizers: dict = {}
        self.extra = setup_fn(self) if setup_fn is not None else None
        self._lock = threading.Lock()
        self._next_seq = 0
        self._pending: dict = {}
        self._q: queue.Queue = queue.Queue()
        self._t = threading.Thread(target=self._run, daemon=True)
        self._t.start()

    def _run(self):
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        while True:
            fn, fut = self._q.get()
            if fn is None:
                return
            try:
                fut.set_result(fn())
            except Exception as exc:  # noqa: BLE001 - shipped back to the caller
                fut.set_exception(exc)

    def submit(self, fn, seq: int | None = None) -> torch.futures.Future:
        """Queue ``fn`` on the executor.  With ``seq`` (assigned by the single driving caller) calls run
        strictly in sequence order even if the RPC agent's thread pool delivers them out of order --
        required so RCCL send/recv pairs of neighbouring stages match."""
        fut = torch.futures.Future()
        if seq is None:
            self._q.put((fn, fut))
            return fut
        with self._lock:
            self._pending[seq] = (fn, fut)
            while self._next_seq in self._pending:
                self._q.put(self._pending.pop(self._next_seq))
                self._next_seq += 1
        return fut

    def stop(self):
        self._q.put((None, None))


def _server(rref_or_id):
    return _SERVERS[rref_or_id] if isinstance(rref_or_id, int) else rref_or_id.local_value()


# --------------------------------------------------------------------------------------------------
# distributed autograd context (master side)
# --------------------------------------------------------------------------------------------------
class _Context:
    _ids = itertools.count(1)

    def __init__(self):
        self.id = next(self._ids)
        self.pending: list = []  # futures of remote backwards
        self.calls = itertools.count()


_CTX = threading.local()


@contextlib.contextmanager
def context():
    """``with dist_autograd.context() as cid:`` (rpc/model_parallel_ResNet50.py:222)."""
    ctx = _Context()
    prev = getattr(_CTX, "ctx", None)
    _CTX.ctx = ctx
    try:
        yield ctx.id
    finally:
        _CTX.ctx = prev
        _CONTEXTS.pop(ctx.id, None)


_CONTEXTS: dict = {}


def current_context() -> _Context:
    ctx = getattr(_CTX, "ctx", None)
    if ctx is None:
        ctx = _Context()  # implicit context (single step)
        _CTX.ctx = ctx
    _CONTEXTS[ctx.id] = ctx
    return ctx


def dist_autograd_backward(context_id, roots):
    """Run backward from ``roots`` locally and wait until every remote backward it triggered is done."""
    ctx = _CONTEXTS.get(context_id) or current_context()
    torch.autograd.backward(roots)
    futs, ctx.pending = ctx.pending, []
    for f in futs:
        f.wait()


class _RemoteCallFn(torch.autograd.Function):
    """Connects a remote call's (CPU) output to the local graph; backward ships grad_output to the owner."""

    @staticmethod
    def forward(ctx, anchor, out, owner_rref, ctx_id, call_id, backward_fn):
        ctx.owner, ctx.ctx_id, ctx.call_id, ctx.backward_fn = owner_rref, ctx_id, call_id, backward_fn
        return out.clone()

    @staticmethod
    def backward(ctx, grad):
        fut = ctx.backward_fn(ctx.owner, ctx.ctx_id, ctx.call_id, grad.contiguous())
        _CONTEXTS[ctx.ctx_id].pending.append(fut)
        return None, None, None, None, None, None


def attach(out: torch.Tensor, owner_rref, ctx: _Context, call_id, backward_fn) -> torch.Tensor:
    anchor = torch.zeros((), requires_grad=True)
    return _RemoteCallFn.apply(anchor, out, owner_rref, ctx.id, call_id, backward_fn)


# --------------------------------------------------------------------------------------------------
# distributed optimizer
# --------------------------------------------------------------------------------------------------
def _remote_make_optimizer(server_rref, opt_cls, opt_kwargs, key):
    srv = server_rref.local_value()
    srv.optimizers[key] = opt_cls([p for p in srv.module.parameters() if p.requires_grad], **opt_kwargs)
    return True


def _remote_step(server_rref, key, ctx_id):
    srv = server_rref.local_value()

    def run():
        grads = srv.grads.pop(ctx_id, None)
        params = [p for p in srv.module.parameters() if p.requires_grad]
        if grads is not None:
            for p in params:
                p.grad = grads.get(p)
        srv.optimizers[key].step()
        for p in params:
            p.grad = None
        if torch.device(srv.device).type == "cuda":
            # the stage's one-launch BatchNorm hand-offs of this step: the master's opt.step() raises on a
            # timeout instead of the stage training on with incomplete statistics (syncs the stage's device;
            # the master waits for this step anyway before the next batch's forward)
            from ..ops.functional import check_device_errors

            check_device_errors(f"stage server {rpc.get_worker_info().name}")
        return True

    return srv.submit(run).wait()


class DistributedOptimizer:
    """``DistributedOptimizer(optim_cls, remote_param_owners, **kw)`` -> one local optimizer per owner.

    ``params`` may be a list of parameter RRefs (the reference's ``parameter_rrefs()``, :180-184) or of
    module-server RRefs; parameters are grouped by owner and each owner gets a fused optimizer over its
    whole module (the reference creates a local optimizer per owner too, via ``_ScriptLocalOptimizer``)."""

    _keys = itertools.count(1)

    def __init__(self, optimizer_class, params, **kwargs):
        from ..ops.optim import FusedAdam, FusedAdamW, FusedSGD

        fused = {torch.optim.SGD: FusedSGD, torch.optim.Adam: FusedAdam, torch.optim.AdamW: FusedAdamW}
        cls = fused.get(optimizer_class, optimizer_class)
        owners = {}
        local = []
        for r in params:
            srv = getattr(r, "_pde_server", None)
            if srv is not None:
                owners[(srv.owner().name, id(srv))] = srv
            elif isinstance(r, rpc.RRef) and r.is_owner():
                local.append(r.local_value())  # a local parameter wrapped in RRef(p) (:78-82)
            elif torch.is_tensor(r):
                local.append(r)
            else:
                raise TypeError("DistributedOptimizer expects parameter_rrefs() / RRef(local_param)")
        self.owners = list(owners.values())
        self.local_opt = cls(local, **kwargs) if local else None
        self.key = next(self._keys)
        futs = [rpc.rpc_async(s.owner(), _remote_make_optimizer, args=(s, cls, kwargs, self.key))
                for s in self.owners]
        for f in futs:
            f.wait()

    def step(self, context_id):
        futs = [rpc.rpc_async(s.owner(), _remote_step, args=(s, self.key, context_id)) for s in self.owners]
        if self.local_opt is not None:
            self.local_opt.step()
            self.local_opt.zero_grad(set_to_none=False)
        for f in futs:
            f.wait()


class ParamRRef:
    """What ``parameter_rrefs()`` returns: names one parameter of a remote module server.  Carries the
    server RRef so :class:`DistributedOptimizer` can group by owner."""

    def __init__(self, server_rref, index):
        self._pde_server = server_rref
        self.index = index

    def owner(self):
        return self._pde_server.owner()


def _remote_num_params(server_rref):
    return sum(1 for p in server_rref.local_value().module.parameters() if p.requires_grad)


def parameter_rrefs(server_rref):
    n = rpc.rpc_sync(server_rref.owner(), _remote_num_params, args=(server_rref,))
    return [ParamRRef(server_rref, i) for i in range(n)]


def accumulate_grads(srv: ModuleServer, ctx_id):
    """Move the module's freshly computed .grad into the per-context store (then clear .grad)."""
    store = srv.grads.setdefault(ctx_id, {})
    for p in srv.module.parameters():
        if p.grad is not None:
            if p in store:
                store[p] += p.grad
            else:
                store[p] = p.grad
            p.grad = None
