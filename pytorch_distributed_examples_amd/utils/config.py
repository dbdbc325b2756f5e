"""Shared run-time configuration for every entry point.

The reference scripts each hard-code their knobs (batch size, lr, bucket cap = DDP's default 25 MiB, fp32
everywhere).  Here the knobs that are common to all workloads live in ONE place, settable per run from the
command line (:func:`add_runtime_args` -- every app calls it, in its own flag style) or the environment (for
launchers that cannot pass flags, e.g. ``hvdrun`` re-launching a worker):

=================  =====================  ==========================================================
flag               environment            meaning
=================  =====================  ==========================================================
``--bucket-mb``    ``PDE_BUCKET_MB``      DDP gradient bucket cap in MiB (default: sized for 7 xGMI
                                          links by :mod:`..parallel.xgmi`)
``--grad-dtype``   ``PDE_GRAD_DTYPE``     gradient wire dtype of the all-reduce: ``fp32`` | ``bf16``
``--dtype``        ``PDE_DTYPE``          compute dtype on the GPU: ``bf16`` (MFMA operands, fp32
                                          accumulate -- the only GPU compute dtype); ``fp32`` = the
                                          CPU reference path
``--seed``         ``PDE_SEED``           torch / synthetic-data seed
``--debug-sync``   ``PDE_DEBUG_SYNC=1``   serialize every native op: synchronize after it and raise
                                          with the op's name on any HIP error (race / fault bisection)
=================  =====================  ==========================================================

Flags win over the environment; unset flags fall back to it, then to the defaults.
"""
from __future__ import annotations

import argparse
import os
from dataclasses import dataclass

import torch


@dataclass
class RuntimeConfig:
    bucket_mb: float | None = None
    grad_dtype: str = "fp32"
    dtype: str = "bf16"
    seed: int = 0
    debug_sync: bool = False

    @property
    def grad_torch_dtype(self):
        return torch.bfloat16 if self.grad_dtype == "bf16" else None

    def ddp_kwargs(self) -> dict:
        """Keyword arguments for :class:`..parallel.ddp.DistributedDataParallel`."""
        return {"bucket_cap_mb": self.bucket_mb, "grad_dtype": self.grad_torch_dtype}


def _flag(style: str, name: str) -> str:
    return "--" + (name.replace("_", "-") if style == "dash" else name)


def add_runtime_args(parser: argparse.ArgumentParser, style: str = "dash") -> argparse.ArgumentParser:
    """Add the shared flags; ``style`` "dash" (``--bucket-mb``) or "underscore" (``--bucket_mb``, the reference
    mnist_ddp_elastic.py's own flag style)."""
    g = parser.add_argument_group("runtime (shared by all entry points; utils/config.py)")
    g.add_argument(_flag(style, "bucket_mb"), dest="bucket_mb", type=float, default=None,
                   help="DDP gradient bucket cap in MiB (default: xGMI-sized)")
    g.add_argument(_flag(style, "grad_dtype"), dest="grad_dtype", choices=["fp32", "bf16"], default=None,
                   help="all-reduce wire dtype (default fp32)")
    g.add_argument(_flag(style, "dtype"), dest="dtype", choices=["bf16", "fp32"], default=None,
                   help="compute dtype: bf16 on the GPU (MFMA, fp32 accumulate); fp32 = CPU reference path")
    g.add_argument(_flag(style, "seed"), dest="seed", type=int, default=None)
    g.add_argument(_flag(style, "debug_sync"), dest="debug_sync", action="store_true", default=None,
                   help="serialize every native op and check HIP errors after it")
    return parser


def from_args(args=None) -> RuntimeConfig:
    """Flags (when given) over ``PDE_*`` environment variables over defaults."""
    def pick(name, env, conv, default):
        v = getattr(args, name, None) if args is not None else None
        if v is not None:
            return v
        e = os.environ.get(env)
        return conv(e) if e not in (None, "") else default

    cfg = RuntimeConfig(
        bucket_mb=pick("bucket_mb", "PDE_BUCKET_MB", float, None),
        grad_dtype=pick("grad_dtype", "PDE_GRAD_DTYPE", str, "fp32"),
        dtype=pick("dtype", "PDE_DTYPE", str, "bf16"),
        seed=pick("seed", "PDE_SEED", int, 0),
        debug_sync=bool(pick("debug_sync", "PDE_DEBUG_SYNC", lambda s: s == "1", False)),
    )
    if cfg.grad_dtype not in ("fp32", "bf16"):
        raise ValueError(f"grad dtype must be fp32 or bf16, got {cfg.grad_dtype!r}")
    if cfg.dtype not in ("fp32", "bf16"):
        raise ValueError(f"compute dtype must be bf16 or fp32, got {cfg.dtype!r}")
    return cfg


def apply(cfg: RuntimeConfig) -> RuntimeConfig:
    """Process-wide effects: seeding and the serialized debug mode of the native ops."""
    torch.manual_seed(cfg.seed)
    if cfg.debug_sync:
        from .. import _native

        _native.set_debug_sync(True)
    return cfg


def device_for(cfg: RuntimeConfig, requested: str) -> str:
    """``--device`` with the compute dtype folded in: fp32 compute is the CPU reference path."""
    if cfg.dtype == "fp32":
        return "cpu"
    return requested
