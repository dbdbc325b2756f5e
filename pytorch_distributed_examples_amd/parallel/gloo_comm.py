"""A gloo stand-in for :class:`_comm.RcclComm` (CPU rehearsal of the elastic re-wire protocol).

``elastic.rewire.RoundComm`` builds its data-plane communicator from a fresh RCCL unique id, by shrinking the
previous round's communicator after a failure, or by splitting it for a planned scale-down.  Those paths run
on GPUs only; with ``PDE_REWIRE_EMULATE=gloo`` the same RoundComm code drives this class instead, so the
decision logic (init / shrink / split, who participates, which ranks leave, rank renumbering) is exercised
by the CPU test suite with real processes.  The interface is the subset RoundComm uses: ``init``,
``split_from`` (collective over every parent rank; ``color < 0`` leaves), ``abort``, ``destroy``, ``valid``,
``rank`` / ``size``, ``async_error``, ``nranks`` and asynchronous all-reduce / broadcast.  Each communicator
is a standalone ``ProcessGroupGloo`` on its own store prefix, independent of the round's control group.
"""
from __future__ import annotations

import datetime
import itertools

import torch
import torch.distributed as dist

_ids = itertools.count()


class GlooComm:
    emulated = True

    def __init__(self):
        self.pg = None
        self.rank, self.size = -1, 0
        self._store = None
        self._prefix = ""
        self._splits = 0

    @staticmethod
    def shrink_supported() -> bool:
        return False  # like torch's bundled RCCL 2.26: no ncclCommShrink

    @property
    def valid(self) -> bool:
        return self.pg is not None

    def init(self, store, prefix: str, rank: int, size: int, timeout_s: float = 60.0):
        self._store, self._prefix = store, prefix
        self.pg = dist.ProcessGroupGloo(dist.PrefixStore(prefix, store), rank, size,
                                        datetime.timedelta(seconds=timeout_s))
        self.rank, self.size = rank, size

    def split_from(self, parent: "GlooComm", color: int, key: int, timeout_s: float = 300.0) -> bool:
        """ncclCommSplit semantics: every parent rank calls; ranks with ``color >= 0`` form the child ordered by
        ``key``; ``color < 0`` gets no communicator (returns False)."""
        if parent.pg is None:
            raise RuntimeError("gloo comm: split from an invalid communicator")
        info = torch.tensor([color, key], dtype=torch.long)
        out = [torch.zeros(2, dtype=torch.long) for _ in range(parent.size)]
        parent.pg.allgather([out], [info]).wait()
        parent._splits += 1
        if color < 0:
            return False
        mine = sorted((int(o[1]), r) for r, o in enumerate(out) if int(o[0]) == color)
        new_rank = [r for _, r in mine].index(parent.rank)
        self.init(parent._store, f"{parent._prefix}/split{parent._splits}/c{color}", new_rank, len(mine))
        return True

    def shrink_from(self, parent: "GlooComm", exclude, abort_parent: bool = True) -> int:
        """ncclCommShrink semantics (survivors only, the excluded ranks do not call): the child keeps the
        parent's rank order minus ``exclude``.  Only reached when ``shrink_supported`` is patched in tests."""
        if parent.pg is None:
            raise RuntimeError("gloo comm: shrink from an invalid communicator")
        keep = [r for r in range(parent.size) if r not in set(exclude)]
        parent._splits += 1
        self.init(parent._store, f"{parent._prefix}/shrink{parent._splits}", keep.index(parent.rank), len(keep))
        return 1

    def abort(self):
        self.pg = None

    def destroy(self):
        self.pg = None

    def async_error(self) -> int:
        return 0 if self.pg is not None else 5  # ncclInvalidUsage

    def nranks(self) -> int:
        return self.size if self.pg is not None else 0

    def allreduce_async(self, t: torch.Tensor, avg: bool = False):
        work = self.pg.allreduce([t])
        if not avg:
            return work

        class _Avg:
            def wait(self_inner):
                work.wait()
                t.div_(self.size)
                return True

        return _Avg()

    def broadcast_(self, t: torch.Tensor, src: int):
        opts = dist.BroadcastOptions()
        opts.rootRank = src
        self.pg.broadcast([t], opts).wait()
        return t
