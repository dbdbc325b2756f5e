"""Elastic rendezvous client: membership rounds published by the elastic driver (launch/hvdrun.py).

The driver hosts a c10d ``TCPStore``; for every membership change it publishes a new *round*:

    round/<r>/size          world size of round r
    round/<r>/rank/<wid>    rank of worker id <wid> in round r (survivors keep their relative order,
                            so rank 0 is always a worker that holds the latest committed state)
    round                   the latest round number (written last)
    updated/<r>             set when hosts were added/removed after round r started
                            (State.commit() -> HostsUpdatedInterrupt)

Workers join round r through ``PrefixStore("pg/<r>", store)``: a fresh process group (gloo) and a
fresh RCCL communicator (unique id under the same prefix) per round, built IN-PROCESS -- this is the
"re-wire without job restart" path.
"""
from __future__ import annotations

import datetime
import os
import time

import torch.distributed as dist


def elastic_env() -> bool:
    return bool(os.environ.get("PDE_ELASTIC_STORE"))


class RendezvousClient:
    def __init__(self, timeout_s: float = 600.0):
        host, port = os.environ["PDE_ELASTIC_STORE"].rsplit(":", 1)
        self.wid = os.environ["PDE_WORKER_ID"]
        self.timeout_s = timeout_s
        self.store = dist.TCPStore(host, int(port), is_master=False,
                                   timeout=datetime.timedelta(seconds=timeout_s), wait_for_workers=False)
        self.round = -1
        self.rank = -1
        self.size = 0

    def _current_round(self) -> int:
        if not self.store.check(["round"]):
            return -1
        return int(self.store.get("round").decode())

    def join(self, after_round: int | None = None):
        """Block until a round newer than ``after_round`` includes this worker; returns (round, rank, size)."""
        after = self.round if after_round is None else after_round
        t0 = time.time()
        while True:
            r = self._current_round()
            if r > after:
                key = f"round/{r}/rank/{self.wid}"
                if self.store.check([key]):
                    self.round = r
                    self.rank = int(self.store.get(key).decode())
                    self.size = int(self.store.get(f"round/{r}/size").decode())
                    return self.round, self.rank, self.size
                if self.store.check(["shutdown"]):
                    raise SystemExit(0)
                if self.round >= 0 and self.store.check([f"round/{r}/members"]):
                    # a member of an earlier round that the newest one drops: the driver removed this worker's
                    # host (planned scale-down; the driver never re-adds a worker id) -> leave cleanly
                    raise SystemExit(0)
            if time.time() - t0 > self.timeout_s:
                raise TimeoutError(f"worker {self.wid}: no rendezvous round after {after} within {self.timeout_s}s")
            time.sleep(0.05)

    def members(self, rnd: int | None = None) -> list[str]:
        """Worker ids of round ``rnd`` (default: the current one) in rank order."""
        r = self.round if rnd is None else rnd
        key = f"round/{r}/members"
        if r < 0 or not self.store.check([key]):
            return []
        return self.store.get(key).decode().split(",")

    def pg_store(self):
        return dist.PrefixStore(f"pg/{self.round}", self.store)

    def hosts_updated(self) -> bool:
        return self.round >= 0 and (self.store.check([f"updated/{self.round}"]) or self._current_round() > self.round)

    def report(self, key: str, value: str):
        self.store.set(f"report/{self.wid}/{key}", value)
