"""Sharded batch loader with DataLoader + DistributedSampler semantics (mnist_ddp_elastic.py:178-189).

For datasets that hold whole tensors (``images``/``labels``, e.g. :class:`SyntheticMNIST` resident in HBM),
batches are built by ONE index gather on the device instead of per-sample collation through worker
processes -- on an MI355X the 188 MB MNIST train set simply lives in HBM.  Sharding and shuffling are
exactly ``torch.utils.data.distributed.DistributedSampler``'s (same seed / epoch semantics, padding to
an equal number of samples per rank), so ``len(loader)`` and per-rank sample sets match the reference.

``start_batch`` skips whole batches without loading them (quirk Q10: the Horovod-elastic reference loads
and discards skipped batches).
"""
from __future__ import annotations

import torch
from torch.utils.data.distributed import DistributedSampler


class ShardedLoader:
    def __init__(self, dataset, batch_size: int, num_replicas: int = 1, rank: int = 0, shuffle: bool = True,
                 seed: int = 0, drop_last: bool = False):
        self.dataset = dataset
        self.batch_size = batch_size
        self.sampler = DistributedSampler(dataset, num_replicas=num_replicas, rank=rank, shuffle=shuffle,
                                          seed=seed, drop_last=drop_last)
        self.start_batch = 0

    def __len__(self):
        n = len(self.sampler)
        return (n + self.batch_size - 1) // self.batch_size

    def set_epoch(self, epoch: int):
        self.sampler.set_epoch(epoch)

    def __iter__(self):
        idx = torch.tensor(list(iter(self.sampler)), dtype=torch.long)
        images, labels = getattr(self.dataset, "images", None), getattr(self.dataset, "labels", None)
        dev = images.device if images is not None else torch.device("cpu")
        idx_dev = idx.to(dev)
        for b in range(self.start_batch, len(self)):
            sl = idx_dev[b * self.batch_size:(b + 1) * self.batch_size]
            if images is not None:
                yield images.index_select(0, sl), labels.index_select(0, sl)
            else:
                items = [self.dataset[int(i)] for i in sl.tolist()]
                yield torch.stack([a for a, _ in items]), torch.as_tensor([b_ for _, b_ in items])
        self.start_batch = 0
