"""RPC-style model parallelism and parameter servers with an RCCL data plane (see :mod:`.core`).

    from pytorch_distributed_examples_amd import rpc as prpc
    with prpc.dist_autograd.context() as cid:
        out = pipeline(inputs)                       # RemotePipeline / RemoteModule calls
        prpc.dist_autograd.backward(cid, [loss_fn(out, labels)])
        opt.step(cid)                                # prpc.DistributedOptimizer
"""
from types import SimpleNamespace

from .core import DistributedOptimizer, ModuleServer, ParamRRef, context, dist_autograd_backward, parameter_rrefs
from .pipeline_rpc import RemotePipeline
from .remote_module import RemoteModule

dist_autograd = SimpleNamespace(context=context, backward=dist_autograd_backward)

__all__ = ["DistributedOptimizer", "ModuleServer", "ParamRRef", "RemoteModule", "RemotePipeline", "context",
           "dist_autograd", "dist_autograd_backward", "parameter_rrefs"]
