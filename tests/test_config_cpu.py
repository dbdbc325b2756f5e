"""Shared run-time configuration (utils/config.py) and the serialized debug mode of the native ops."""
import argparse

import pytest

from pytorch_distributed_examples_amd import _native
from pytorch_distributed_examples_amd.utils import config


def test_flags_over_env_over_defaults(monkeypatch):
    monkeypatch.setenv("PDE_BUCKET_MB", "4")
    monkeypatch.setenv("PDE_GRAD_DTYPE", "bf16")
    ap = config.add_runtime_args(argparse.ArgumentParser(), style="underscore")
    cfg = config.from_args(ap.parse_args([]))
    assert cfg.bucket_mb == 4.0 and cfg.grad_dtype == "bf16" and cfg.dtype == "bf16" and not cfg.debug_sync
    cfg = config.from_args(ap.parse_args(["--bucket_mb", "1.5", "--grad_dtype", "fp32", "--debug_sync"]))
    assert cfg.bucket_mb == 1.5 and cfg.grad_dtype == "fp32" and cfg.debug_sync
    assert cfg.ddp_kwargs() == {"bucket_cap_mb": 1.5, "grad_dtype": None}
    ap2 = config.add_runtime_args(argparse.ArgumentParser(), style="dash")
    cfg = config.from_args(ap2.parse_args(["--grad-dtype", "bf16", "--dtype", "fp32", "--seed", "7"]))
    import torch

    assert cfg.ddp_kwargs()["grad_dtype"] is torch.bfloat16 and cfg.seed == 7
    assert config.device_for(cfg, "gpu") == "cpu"  # fp32 compute = the CPU reference path
    monkeypatch.setenv("PDE_GRAD_DTYPE", "fp8")
    with pytest.raises(ValueError):
        config.from_args(None)


def test_ddp_takes_bucket_cap_from_config():
    import torch

    from pytorch_distributed_examples_amd.parallel.ddp import DistributedDataParallel

    m = torch.nn.Sequential(torch.nn.Linear(512, 512), torch.nn.Linear(512, 512))
    cfg = config.RuntimeConfig(bucket_mb=0.5)
    ddp = DistributedDataParallel(m, **cfg.ddp_kwargs())
    assert sum(ddp.bucket_bytes) == sum(p.numel() * 4 for p in m.parameters())


def test_debug_sync_wrapper_checks_every_call(monkeypatch):
    calls = []

    class FakeMod:
        def op(self, x):
            calls.append(("op", x))
            return x + 1

        def clear_last_error(self):
            calls.append(("err",))
            return 0

    import torch

    monkeypatch.setattr(torch.cuda, "is_available", lambda: False)  # CPU: no synchronize, call passes through
    w = _native._SyncChecked(FakeMod())
    assert w.op(1) == 2 and calls == [("op", 1)]
