"""Snapshot checkpoint compatible with the reference's format (pytorch_elastic/mnist_ddp_elastic.py:95-104).

``{"MODEL_STATE": module.state_dict(), "EPOCHS_RUN": epoch}`` -- the same keys, so snapshots move
between the reference and this suite.  Deliberate fixes:

* written by GLOBAL rank 0 only (the reference writes from every node's local rank 0, racing on a
  shared path), through a temp file + ``os.replace`` so a crash mid-write never leaves a torn file;
* optional ``OPTIMIZER_STATE`` (the reference drops optimizer state); loaders accept snapshots with or
  without it;
* resume semantics are kept: ``EPOCHS_RUN`` is the epoch that was saved, and training restarts AT that
  epoch (the reference re-runs it, Q4) unless ``resume_next=True``.
* loading uses ``torch.load(weights_only=True)`` -- nothing in the file is executed.
"""
from __future__ import annotations

import os
import tempfile

import torch


def _to_cpu(obj):
    if torch.is_tensor(obj):
        return obj.detach().cpu()
    if isinstance(obj, dict):
        return {k: _to_cpu(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_cpu(v) for v in obj)
    return obj


def save_snapshot(path: str, model_state: dict, epochs_run: int, optimizer_state: dict | None = None) -> None:
    snap = {"MODEL_STATE": _to_cpu(model_state), "EPOCHS_RUN": int(epochs_run)}
    if optimizer_state is not None:
        snap["OPTIMIZER_STATE"] = _to_cpu(optimizer_state)
    d = os.path.dirname(os.path.abspath(path)) or "."
    os.makedirs(d, exist_ok=True)
    fd, tmp = tempfile.mkstemp(prefix=".snapshot.", dir=d)
    try:
        with os.fdopen(fd, "wb") as f:
            torch.save(snap, f)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, path)
    except BaseException:
        if os.path.exists(tmp):
            os.unlink(tmp)
        raise


def load_snapshot(path: str, map_location="cpu") -> dict:
    snap = torch.load(path, map_location=map_location, weights_only=True)
    if "MODEL_STATE" not in snap or "EPOCHS_RUN" not in snap:
        raise ValueError(f"{path} is not a snapshot (needs MODEL_STATE and EPOCHS_RUN)")
    return snap
