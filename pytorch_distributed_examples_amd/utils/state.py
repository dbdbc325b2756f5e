"""Deep copies of training state (state_dicts: nested dicts / lists of tensors) for in-memory commits --
``hvd.elastic.TorchState.commit`` and the in-process re-wire's round commits (``elastic.rewire``)."""
from __future__ import annotations

import copy

import torch


def clone_state(obj):
    """Tensors detached and cloned on their device; containers rebuilt with their own type; anything else
    deep-copied."""
    if torch.is_tensor(obj):
        return obj.detach().clone()
    if isinstance(obj, dict):
        return type(obj)((k, clone_state(v)) for k, v in obj.items())
    if isinstance(obj, (list, tuple)):
        return type(obj)(clone_state(v) for v in obj)
    return copy.deepcopy(obj)
