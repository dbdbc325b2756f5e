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
