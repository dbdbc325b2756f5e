"""Loader for the in-tree native extensions (``_C`` kernels, ``_comm`` runtime).

GPU code paths call :func:`C` / :func:`comm`; if the extension is missing or fails to load they raise
immediately (no silent eager fallback on a GPU box).  CPU-only code paths never touch these modules.
Set ``PDE_AUTOBUILD=1`` to compile on first use (hipcc for gfx950 is available in the build image).
"""
from __future__ import annotations

import importlib
import os

_mods: dict[str, object] = {}
_DEBUG_SYNC = [os.environ.get("PDE_DEBUG_SYNC", "0") == "1"]


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


class _SyncChecked:
    """Debug view of a native module (``PDE_DEBUG_SYNC=1`` / ``--debug-sync``): every call is
    followed by a device synchronize and a HIP last-error check that raises with the op's name, so an
    asynchronous fault, an out-of-bounds access or a missing stream dependency is pinned to the launch that
    caused it instead of surfacing at some later synchronization.  Inside a stream capture the checks are
    skipped (synchronizing would invalidate the capture)."""

    def __init__(self, mod):
        self._mod = mod

    def __getattr__(self, name):
        fn = getattr(self._mod, name)
        if not callable(fn) or name in ("clear_last_error",):
            return fn
        mod = self._mod

        def checked(*a, **k):
            out = fn(*a, **k)
            import torch

            if torch.cuda.is_available() and not torch.cuda.is_current_stream_capturing():
                torch.cuda.synchronize()
                err = mod.clear_last_error() if hasattr(mod, "clear_last_error") else 0
                if err:
                    raise RuntimeError(f"native op {name!r} left HIP error {err} (PDE_DEBUG_SYNC)")
            return out

        return checked


def set_debug_sync(flag: bool) -> None:
    _DEBUG_SYNC[0] = bool(flag)


def debug_sync() -> bool:
    return _DEBUG_SYNC[0]


def C():
    """The gfx950 kernel extension (GEMM/conv/BN/pool/loss/optimizer/...)."""
    mod = _load("_C")
    return _SyncChecked(mod) if _DEBUG_SYNC[0] else mod


def comm():
    """The native communication runtime (RCCL communicator manager, fusion engine)."""
    return _load("_comm")


def loaded(name: str = "_C") -> bool:
    """Whether the extension was already loaded by this process (no import attempted)."""
    return name in _mods


def available(name: str = "_C") -> bool:
    try:
        _load(name)
        return True
    except NativeUnavailable:
        return False
