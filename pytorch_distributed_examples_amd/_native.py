"""Loader for the in-tree native extensions (``_C`` kernels, ``_comm`` runtime).

GPU code paths call :func:`C` / :func:`comm`; if the extension is missing or fails to load they raise
immediately (no silent eager fallback on a GPU box).  CPU-only code paths never touch these modules.
Set ``PDE_AUTOBUILD=1`` to compile on first use (hipcc for gfx950 is available in the build image).
"""
from __future__ import annotations

import importlib
import os

_mods: dict[str, object] = {}


class NativeUnavailable(RuntimeError):
    pass


def _load(name: str):
    if name in _mods:
        return _mods[name]
    try:
        mod = importlib.import_module(f"pytorch_distributed_examples_amd.{name}")
    except ImportError as exc:
        if os.environ.get("PDE_AUTOBUILD", "0") == "1":
            from . import _build

            _build.build()
            mod = importlib.import_module(f"pytorch_distributed_examples_amd.{name}")
        else:
            raise NativeUnavailable(
                f"native extension pytorch_distributed_examples_amd.{name} is not built "
                f"(run `python -m pytorch_distributed_examples_amd._build`): {exc}") from exc
    _mods[name] = mod
    return mod


def C():
    """The gfx950 kernel extension (GEMM/conv/BN/pool/loss/optimizer/...)."""
    return _load("_C")


def comm():
    """The native communication runtime (RCCL communicator manager, fusion engine)."""
    return _load("_comm")


def available(name: str = "_C") -> bool:
    try:
        _load(name)
        return True
    except NativeUnavailable:
        return False
