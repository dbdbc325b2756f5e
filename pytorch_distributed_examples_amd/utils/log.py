"""Rank-aware logging and JSONL metrics (the reference only has bare ``print``)."""
from __future__ import annotations

import json
import sys
import time


class RankLogger:
    """``print`` that defaults to rank 0 and can prefix the rank; keeps the reference's message text."""

    def __init__(self, rank: int = 0, prefix: bool = False, stream=None):
        self.rank = rank
        self.prefix = prefix
        self.stream = stream or sys.stdout

    def print(self, msg: str, all_ranks: bool = False):
        if all_ranks or self.rank == 0:
            text = f"[rank {self.rank}] {msg}" if self.prefix else msg
            print(text, file=self.stream, flush=True)


class MetricsWriter:
    """Append one JSON object per call (images/s, step time, loss, ...)."""

    def __init__(self, path: str):
        self.path = path

    def write(self, **fields):
        fields.setdefault("ts", time.time())
        with open(self.path, "a") as f:
            f.write(json.dumps(fields) + "\n")


class StepTimer:
    """Accumulates named phase times (fwd / bwd / comm / optim); GPU phases should be synchronized by
    the caller or measured with events."""

    def __init__(self):
        self.totals: dict[str, float] = {}
        self._t = None
        self._name = None

    def start(self, name: str):
        self.stop()
        self._name, self._t = name, time.perf_counter()

    def stop(self):
        if self._name is not None:
            self.totals[self._name] = self.totals.get(self._name, 0.0) + time.perf_counter() - self._t
            self._name = None


class PhaseTimer:
    """Per-phase device time of eager steps (fwd / bwd / comm wait / optimizer, and per
    pipeline stage: forward / backward compute and the time a stage's stream spends in receive waits).

    ``with timer.phase("fwd"): ...`` records a HIP event pair on the current stream around the work (on
    CPU: wall time); :meth:`summary` synchronises once and returns milliseconds per phase, summed over the
    recorded steps and divided by ``steps``.  A captured hipGraph has no host-visible phase boundaries, so
    the bench measures phases on a few eager steps after its timed region."""

    def __init__(self, device=None):
        import torch

        self.cuda = device is not None and torch.device(device).type == "cuda"
        self.marks: list = []
        self.steps = 0

    def phase(self, name: str):
        import contextlib

        import torch

        @contextlib.contextmanager
        def cm():
            if self.cuda:
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                yield
                e.record()
                self.marks.append((name, s, e))
            else:
                t0 = time.perf_counter()
                yield
                self.marks.append((name, t0, time.perf_counter()))

        return cm()

    def summary(self) -> dict:
        import torch

        if self.cuda:
            torch.cuda.synchronize()
        out: dict[str, float] = {}
        for name, s, e in self.marks:
            ms = s.elapsed_time(e) if self.cuda else (e - s) * 1e3
            out[name] = out.get(name, 0.0) + ms
        n = max(1, self.steps)
        return {k: round(v / n, 4) for k, v in out.items()}


class _NoPhase:
    def phase(self, name: str):
        import contextlib

        return contextlib.nullcontext()


NO_PHASES = _NoPhase()
