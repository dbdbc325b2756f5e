"""Epochs of an entry script as hipGraph replays with no per-step host work.

The reference trainers loop ``for source, targets in train_data: _run_batch(...)``
(pytorch_elastic/mnist_ddp_elastic.py:90-91, horovod/mnist_horovod.py:58-67, horovod_mnist_elastic.py:62-75).  On
an MI355X one MNIST step is 30-130 us of GPU time, so a per-step Python iteration -- a DataLoader gather, the copy
into a graph's static inputs, the replay call, a ``loss.item()`` every few batches -- costs as much as the step.
Here an epoch is:

* :class:`EpochBatches`: this rank's ``DistributedSampler`` shard of an HBM-resident dataset, gathered ONCE per epoch
  (one ``index_select`` per tensor) into buffers at fixed addresses; batch ``b`` is a contiguous slice of them --
  the same samples in the same order as :class:`..data.loader.ShardedLoader` (DistributedSampler semantics);
* :class:`ChunkedGraphs`: ``chunk`` consecutive full batches per hipGraph (:class:`.graph.CapturedSteps`, each step
  reading its slice in place), captured once on first use and replayed every epoch -- one host call per chunk.
  Steps before the first capture (``eager_first``), a resumed position inside a chunk and the short last batch run
  eagerly through the same step function;
* :class:`AsyncLossLog`: the reference's per-batch loss prints without a device sync -- each chunk's losses are
  copied to pinned host memory behind an event and printed once the event has fired.

Every captured step is the same complete training step as the eager one (forward, backward, all-reduce, optimiser
update); nothing is skipped or cached.
"""
from __future__ import annotations

import torch


def sampler_indices(s) -> torch.Tensor:
    """``list(iter(s))`` of a ``DistributedSampler`` as one int64 tensor, computed with tensor ops (the Python list of
    60k indices costs ~10 ms per epoch -- several epochs' worth of GPU time for the MNIST nets): same seed / epoch
    permutation, padding and rank stride as torch.utils.data.distributed.DistributedSampler.__iter__."""
    n = len(s.dataset)
    if s.shuffle:
        g = torch.Generator()
        g.manual_seed(s.seed + s.epoch)
        idx = torch.randperm(n, generator=g)
    else:
        idx = torch.arange(n)
    if not s.drop_last:
        pad = s.total_size - n
        if pad > 0:
            idx = torch.cat([idx, idx.repeat(-(-pad // n))[:pad]])
    else:
        idx = idx[:s.total_size]
    return idx[s.rank:s.total_size:s.num_replicas].contiguous()


class EpochBatches:
    """Fixed-address, per-epoch permuted copy of one rank's shard of a whole-tensor dataset (``images``/``labels``)."""

    def __init__(self, loader):
        self.loader = loader
        ds = loader.dataset
        self.images, self.labels = ds.images, ds.labels
        self.batch_size = loader.batch_size
        n = len(loader.sampler)
        self.n = n
        self.x = torch.empty((n,) + tuple(self.images.shape[1:]), dtype=self.images.dtype, device=self.images.device)
        self.y = torch.empty((n,) + tuple(self.labels.shape[1:]), dtype=self.labels.dtype, device=self.labels.device)
        self._last = None
        self._ready: dict = {}  # epoch -> its permutation, computed ahead (prepare)

    def __len__(self) -> int:
        return len(self.loader)

    @property
    def full_batches(self) -> int:
        return self.n // self.batch_size

    def fill(self, epoch: int | None = None) -> None:
        """Gather this epoch's shard (``set_epoch`` first when ``epoch`` is given; the Horovod scripts never call
        it, quirk Q8: their permutation repeats and the gather is skipped)."""
        if epoch is not None:
            self.loader.set_epoch(epoch)
        order = self._ready.pop(self.loader.sampler.epoch, None)
        self._ready.clear()
        if order is None:
            order = sampler_indices(self.loader.sampler)
        if self._last is not None and torch.equal(order, self._last):
            return
        if self.images.is_cuda:
            idx = (order if order.is_pinned() else order.pin_memory()).to(self.images.device, non_blocking=True)
        else:
            idx = order
        torch.index_select(self.images, 0, idx, out=self.x)
        torch.index_select(self.labels, 0, idx, out=self.y)
        self._last = order

    def prepare(self, epoch: int) -> None:
        """Compute epoch ``epoch``'s permutation now (host work: call it while the GPU runs the current epoch)."""
        s = self.loader.sampler
        cur = s.epoch
        s.set_epoch(epoch)
        try:
            self._ready[epoch] = sampler_indices(s).pin_memory() if self.images.is_cuda else sampler_indices(s)
        finally:
            s.set_epoch(cur)

    def batch(self, b: int):
        B = self.batch_size
        return self.x[b * B:(b + 1) * B], self.y[b * B:(b + 1) * B]


class AsyncLossLog:
    """Deferred per-batch loss lines: ``add(batch_indices, loss_tensors)`` after the kernels were enqueued, lines are
    printed by :meth:`poll` once their values reached host memory (no ``.item()`` sync in the loop)."""

    def __init__(self, fmt, every: int, enabled: bool = True):
        self.fmt, self.every, self.enabled = fmt, max(1, int(every)), enabled
        self._q = []

    def add(self, batches, losses):
        if not self.enabled:
            return
        sel = [(b, l) for b, l in zip(batches, losses) if b % self.every == 0 and l is not None]
        if not sel:
            return
        vals = torch.stack([l.detach().reshape(()).float() for _, l in sel])
        host = torch.empty(vals.shape, dtype=torch.float32, pin_memory=vals.is_cuda)
        host.copy_(vals, non_blocking=True)
        ev = None
        if vals.is_cuda:
            ev = torch.cuda.Event()
            ev.record()
        self._q.append((ev, host, [b for b, _ in sel]))
        self.poll()

    def poll(self, wait: bool = False):
        while self._q:
            ev, host, bs = self._q[0]
            if ev is not None and not ev.query():
                if not wait:
                    return
                ev.synchronize()
            self._q.pop(0)
            for b, v in zip(bs, host.tolist()):
                print(self.fmt(b, v), flush=True)


class ChunkedGraphs:
    """Run an epoch's batches through ``step_fn(x, y) -> loss``: full chunks as one hipGraph replay each.

    ``eager_first``: steps run eagerly before the first capture (lazy initialisation, an engine's negotiation).
    ``on_steps(batch_indices, losses)`` is called after every replay / eager step (fault hooks, loss logs)."""

    def __init__(self, step_fn, batches: EpochBatches, chunk: int = 50, eager_first: int = 1, enabled: bool = True,
                 tail_step=None):
        self.step_fn = step_fn
        self.tail_step = tail_step or step_fn  # for the short last batch (a kernel with batch-size constraints)
        self.eb = batches
        self.chunk = max(1, int(chunk))
        self.eager_first = int(eager_first)
        self.enabled = enabled and torch.cuda.is_available() and batches.x.is_cuda
        self.graphs: dict = {}
        self.eager_steps = 0
        self.replays = 0
        self.captures = 0
        self._pool = None

    def _chunk_at(self, b: int):
        """(start, length) of the graph chunk starting at batch ``b``, or None when ``b`` is not a chunk start."""
        nf = self.eb.full_batches
        if b % self.chunk or b >= nf:
            return None
        return b, min(self.chunk, nf - b)

    def _graph(self, start: int, length: int):
        key = (start, length)
        g = self.graphs.get(key)
        if g is None:
            from .graph import CapturedSteps

            if self._pool is None:
                self._pool = torch.cuda.graph_pool_handle()  # chunks never replay concurrently: one pool
            torch.cuda.synchronize()
            g = CapturedSteps(self.step_fn, [self.eb.batch(start + j) for j in range(length)], warmup=0,
                              pool=self._pool).capture()
            self.graphs[key] = g
            self.captures += 1
        return g

    def invalidate(self):
        """Drop every graph (a membership change baked a communicator / world size into them)."""
        self.graphs = {}
        self._pool = None
        self.eager_steps = 0

    def run(self, start: int = 0, stop: int | None = None, on_steps=None):
        """Batches [start, stop) of the current epoch (``EpochBatches.fill`` first); returns (images, last loss)."""
        stop = len(self.eb) if stop is None else min(stop, len(self.eb))
        b, n, loss = start, 0, None
        B = self.eb.batch_size
        while b < stop:
            ch = self._chunk_at(b) if (self.enabled and self.eager_steps >= self.eager_first) else None
            if ch is not None and b + ch[1] <= stop:
                g = self._graph(*ch)
                g.graph.replay()
                self.replays += 1
                outs = g.outputs
                idxs = list(range(b, b + ch[1]))
                b += ch[1]
                n += ch[1] * B
                loss = outs[-1]
            else:
                x, y = self.eb.batch(b)
                fn = self.step_fn if x.shape[0] == B else self.tail_step
                loss = fn(x, y)
                self.eager_steps += 1
                outs, idxs = [loss], [b]
                b += 1
                n += x.shape[0]
            if on_steps is not None:
                on_steps(idxs, outs)
        return n, loss
