"""Environment-driven fault injector for elasticity tests (the reference has none;
faults were injected by hand with ``kill``).

    PDE_FAULT_AT_STEP=k     global step at which to fault (required to arm)
    PDE_FAULT_RANK=r        rank that faults (default 0)
    PDE_FAULT_MODE=exit|sigkill|hang|raise   (default exit)
    PDE_FAULT_ONCE=/path    marker file: fault only if it does not exist yet (created when firing), so a
                            restarted worker group runs through

``raise`` raises :class:`InjectedFault` (a recoverable in-process error, like Horovod's
``HorovodInternalError``) instead of terminating the process.
"""
from __future__ import annotations

import os
import signal
import sys
import time


class InjectedFault(RuntimeError):
    pass


def _armed():
    step = os.environ.get("PDE_FAULT_AT_STEP")
    if step in (None, ""):
        return None
    return int(step), int(os.environ.get("PDE_FAULT_RANK", "0")), os.environ.get("PDE_FAULT_MODE", "exit")


def maybe_fault(step: int, rank: int) -> None:
    maybe_fault_in(step, step + 1, rank)


def maybe_fault_in(lo: int, hi: int, rank: int) -> None:
    """Fault if the armed step lies in ``[lo, hi)`` -- for loops that advance several steps at once (a hipGraph
    replay of G training steps): the fault fires after the replay that contains the armed step."""
    cfg = _armed()
    if cfg is None:
        return
    at, frank, mode = cfg
    if not (lo <= at < hi) or rank != frank:
        return
    step = at
    marker = os.environ.get("PDE_FAULT_ONCE")
    if marker:
        if os.path.exists(marker):
            return
        with open(marker, "w") as f:  # t=: wall clock of the fault (survivors report their detection latency)
            f.write(f"rank {rank} step {step} mode {mode} t={time.time():.6f}\n")
    print(f"[fault-injector] rank {rank} step {step}: {mode}", flush=True)
    if mode == "exit":
        sys.stdout.flush()
        os._exit(17)
    if mode == "sigkill":
        os.kill(os.getpid(), signal.SIGKILL)
    if mode == "hang":
        while True:
            time.sleep(3600)
    raise InjectedFault(f"injected fault at step {step} on rank {rank}")
