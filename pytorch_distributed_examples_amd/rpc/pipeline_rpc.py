"""RPC-driven micro-batched pipeline (rpc/model_parallel_ResNet50.py:142-184 programming model).

A master process holds :class:`RemotePipeline` = remote stage servers on the stage workers.  For every
micro-batch the master issues asynchronous forward calls to all stages (like ``p1_rref.remote().forward``
/ ``p2_rref.rpc_async().forward``, :173-174); stage k receives its input from stage k-1 over RCCL (GPU) --
not by ``to_here()`` -- so the only bytes crossing the RPC agent are the master's input micro-batch and
the last stage's m x 1000 output.  The returned outputs are attached to the master's autograd graph;
``dist_autograd_backward`` ships their gradients back and each stage runs its local backward, passing
activation gradients upstream over RCCL.  Stage servers execute in master-assigned sequence order.

Stage workers form their own process group (RCCL on GPUs, gloo on CPU) for the P2P data plane, exactly
like the reference's hybrid example builds a trainer-only group next to the RPC agent
(rpc/server_model_data_parallel.py:155-166).
"""
from __future__ import annotations

import itertools
import os

import torch
import torch.distributed as dist
import torch.distributed.rpc as rpc

from ..ops import functional as OF
from ..parallel.pipeline import P2PChannel
from . import core


def _stage_setup(stage: int, num_stages: int):
    def setup(srv: core.ModuleServer):
        ch = {"prev": None, "next": None, "meta": None, "sent_meta": False}
        me = dist.get_rank()
        pairs = []
        if stage > 0:
            pairs.append(("prev", me - 1))
        if stage < num_stages - 1:
            pairs.append(("next", me + 1))
        for which, peer in sorted(pairs, key=lambda p: min(p[1], me)):
            ch[which] = P2PChannel(peer, "rpcpipe", srv.device)
        ch["stage"], ch["num_stages"] = stage, num_stages
        return ch

    return setup


def _make_stage_server(module_fn, args, kwargs, device, stage, num_stages):
    return core.ModuleServer(module_fn, args, kwargs, device, setup_fn=_stage_setup(stage, num_stages))


@rpc.functions.async_execution
def _stage_forward(srv_rref, ctx_id, call_id, seq, x_cpu, groups=1):
    srv = srv_rref.local_value()
    ch = srv.extra

    def run():
        last = ch["stage"] == ch["num_stages"] - 1
        if ch["prev"] is None:
            x = x_cpu.to(srv.device, non_blocking=False)
        else:
            if ch["meta"] is None:
                ch["meta"] = ch["prev"].recv_meta()
            x = ch["prev"].recv(*ch["meta"]).requires_grad_(True)
        with OF.bn_groups(groups):  # a unit of `groups` micro-batches: per-micro-batch BatchNorm statistics
            y = srv.module(x)
        srv.saved[(ctx_id, call_id)] = (x, y)
        if last:
            return y.detach().float().cpu()
        if not ch["sent_meta"]:
            ch["next"].send_meta(y)
            ch["sent_meta"] = True
        ch["next"].send(y.detach())
        return None

    return srv.submit(run, seq)


@rpc.functions.async_execution
def _stage_backward(srv_rref, ctx_id, call_id, seq, grad_cpu):
    srv = srv_rref.local_value()
    ch = srv.extra

    def run():
        x, y = srv.saved.pop((ctx_id, call_id))
        if grad_cpu is not None:
            g = grad_cpu.to(srv.device).to(y.dtype)
        else:
            g = ch["next"].recv(y.shape, y.dtype)
        torch.autograd.backward(y, g)
        core.accumulate_grads(srv, ctx_id)
        if ch["prev"] is not None:
            ch["prev"].send(x.grad)
        return True

    return srv.submit(run, seq)


class RemotePipeline:
    """Micro-batched pipeline of remote stage modules driven from the master.

    ``stage_fns[i]`` builds stage i on ``workers[i]`` (device ``devices[i]``); ``split_size`` is the
    micro-batch SIZE (the reference's ``split_size`` semantics, quirk Q2)."""

    def __init__(self, split_size: int, workers, stage_fns, devices, stage_args=None, mb_group: int | None = None):
        self.split_size = split_size
        # micro-batches per pipeline unit (grouped BatchNorm keeps per-micro-batch statistics; see
        # apps/hybrid_ps.ResNetPipelineDP): default all of them when the stages run on GPUs
        if mb_group is None:
            env = os.environ.get("PDE_PIPE_MB_GROUP")
            mb_group = int(env) if env else (0 if any(torch.device(d).type == "cuda" for d in devices) else 1)
        self.mb_group = mb_group  # 0: every micro-batch of the batch in one unit
        self.workers = list(workers)
        n = len(self.workers)
        stage_args = stage_args or [() for _ in range(n)]
        futs = [rpc.remote(w, _make_stage_server, args=(fn, a, {}, d, i, n))
                for i, (w, fn, d, a) in enumerate(zip(self.workers, stage_fns, devices, stage_args))]
        self.stages = futs  # RRefs to ModuleServer (construction runs concurrently -> P2P rendezvous)
        for r in self.stages:
            r._get_future().wait()  # constructed (the server itself is not picklable: never to_here())
        self._seq = [itertools.count() for _ in self.stages]

    def _call(self, i, fn, *args):
        return rpc.rpc_async(self.workers[i], fn, args=(self.stages[i],) + args[:2] + (next(self._seq[i]),) + args[2:])

    def forward(self, xs: torch.Tensor) -> torch.Tensor:
        ctx = core.current_context()
        outs = []
        n_mb = -(-xs.shape[0] // self.split_size)
        g = n_mb if self.mb_group <= 0 else min(self.mb_group, n_mb)
        while n_mb % g or (g > 1 and xs.shape[0] % self.split_size):  # equal units (whole micro-batches)
            g -= 1
        for x in xs.split(self.split_size * g, dim=0):
            call = next(ctx.calls)
            futs = [self._call(i, _stage_forward, ctx.id, call, x if i == 0 else None, g)
                    for i in range(len(self.stages))]
            outs.append((call, futs[-1]))
        results = []
        for call, f in outs:
            y = f.wait()
            results.append(core.attach(y, None, ctx, call, self._backward_fn))
        return torch.cat(results)

    __call__ = forward

    def _backward_fn(self, _owner, ctx_id, call_id, grad):
        n = len(self.stages)
        futs = [self._call(i, _stage_backward, ctx_id, call_id, grad if i == n - 1 else None)
                for i in reversed(range(n))]
        return torch.futures.collect_all(futs)

    def parameter_rrefs(self):
        rrefs = []
        for s in self.stages:
            rrefs.extend(core.parameter_rrefs(s))
        return rrefs
