"""``broadcast_parameters`` / ``broadcast_optimizer_state`` (horovod/torch/functions.py semantics).

Used by the reference at horovod/mnist_horovod.py:56 and implicitly by elastic ``state.sync()``.
All tensors are broadcast asynchronously through the engine and waited together.
"""
from __future__ import annotations

import collections

import torch

from . import core


def broadcast_parameters(params, root_rank: int = 0):
    """Broadcast a ``state_dict`` (or ``named_parameters()`` list / list of (name, tensor)) from root."""
    if isinstance(params, dict):
        items = sorted(params.items())
    elif isinstance(params, list) or hasattr(params, "__iter__"):
        items = list(params)
        if items and not isinstance(items[0], tuple):
            items = [(f"param.{i}", p) for i, p in enumerate(items)]
    else:
        raise ValueError(f"invalid params of type {type(params)}")
    if core.size() == 1:
        return
    handles = []
    for name, p in items:
        if p is None:
            continue
        t = p.data if isinstance(p, torch.nn.Parameter) else p
        if not torch.is_tensor(t):
            continue
        handles.append(core.broadcast_async_(t, root_rank, name=f"bcast.{name}"))
    for h in handles:
        core.synchronize(h)


def broadcast_optimizer_state(optimizer, root_rank: int = 0):
    """Broadcast optimizer hyper-parameters and state (creating empty state on non-root ranks first)."""
    if core.size() == 1:
        return
    # make sure every rank has materialised state tensors with the root's structure
    sd = optimizer.state_dict()
    root_sd = core.broadcast_object(_structure(sd), root_rank)
    if core.rank() != root_rank:
        _materialise(optimizer, root_sd)
        sd = optimizer.state_dict()
    # hyper-parameters (scalars) travel as an object, tensors through the engine
    groups = core.broadcast_object([{k: v for k, v in g.items() if k != "params"} for g in sd["param_groups"]],
                                   root_rank)
    for g, hp in zip(optimizer.param_groups, groups):
        g.update(hp)
    handles = []
    scalars = {}
    for pid, st in sorted(optimizer.state_dict()["state"].items()):
        for k, v in sorted(st.items()):
            if torch.is_tensor(v) and v.dim() > 0:
                handles.append(core.broadcast_async_(v, root_rank, name=f"opt.{pid}.{k}"))
            else:
                scalars[(pid, k)] = v.item() if torch.is_tensor(v) else v
    for h in handles:
        core.synchronize(h)
    scalars = core.broadcast_object(scalars, root_rank)
    params = [p for g in optimizer.param_groups for p in g["params"]]
    for (pid, k), v in scalars.items():
        p = params[pid]
        cur = optimizer.state[p].get(k)
        if torch.is_tensor(cur):
            cur.fill_(v)
        else:
            optimizer.state[p][k] = v


def _structure(sd):
    return {pid: {k: (tuple(v.shape), str(v.dtype)) if torch.is_tensor(v) else v for k, v in st.items()}
            for pid, st in sd["state"].items()}


def _materialise(optimizer, structure):
    params = [p for g in optimizer.param_groups for p in g["params"]]
    for pid, st in structure.items():
        p = params[pid]
        cur = optimizer.state[p]
        for k, v in st.items():
            if isinstance(v, tuple) and len(v) == 2 and isinstance(v[1], str) and v[1].startswith("torch."):
                if k not in cur:
                    dtype = getattr(torch, v[1].split(".")[1])
                    cur[k] = torch.zeros(v[0], dtype=dtype, device=p.device)
            elif k not in cur:
                cur[k] = v
    return collections.OrderedDict()
