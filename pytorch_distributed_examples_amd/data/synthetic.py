"""Synthetic datasets (no network, no torchvision -- SURVEY.md §7.4 H7, quirk Q7).

* :class:`SyntheticMNIST` -- MNIST-shaped (1x28x28, 10 classes, 60k train / 10k test), normalised like
  the reference's ``transforms.Normalize((0.1307,), (0.3081,))`` (mnist_ddp_elastic.py:166-169).  Each
  class is a fixed random stroke template plus per-sample noise, so the task is learnable and loss /
  accuracy move like they would on MNIST.  Tensors can live on the GPU (one HBM-resident copy; batches
  are index gathers) or be served through a ``torch.utils.data.Dataset`` + ``DistributedSampler`` like
  the reference's DataLoader pipeline.
* :func:`resnet_batch` -- ``randn(B,3,128,128)`` inputs and one-hot targets
  (model_parallel_ResNet50.py:208-217).
* :func:`embbag_batches` -- the random EmbeddingBag batches of server_model_data_parallel.py:49-68
  (quirk Q1 fixed: takes an optional rank used to seed).
"""
from __future__ import annotations

import random

import torch
from torch.utils.data import Dataset

MNIST_MEAN, MNIST_STD = 0.1307, 0.3081


class SyntheticMNIST(Dataset):
    def __init__(self, n: int = 60000, device="cpu", seed: int = 0, classes: int = 10, noise: float = 0.35):
        g = torch.Generator().manual_seed(seed)
        templates = (torch.rand(classes, 1, 28, 28, generator=g) > 0.78).float()
        labels = torch.randint(0, classes, (n,), generator=g)
        # generate in chunks to bound host memory
        imgs = torch.empty(n, 1, 28, 28)
        for s in range(0, n, 8192):
            e = min(n, s + 8192)
            x = templates[labels[s:e]] + noise * torch.randn(e - s, 1, 28, 28, generator=g)
            imgs[s:e] = (x.clamp_(0, 1) - MNIST_MEAN) / MNIST_STD
        self.images = imgs.to(device)
        self.labels = labels.to(device)

    def __len__(self):
        return self.labels.shape[0]

    def __getitem__(self, i):
        return self.images[i], self.labels[i]

    def batch(self, step: int, batch_size: int, rank: int = 0, world: int = 1):
        """Device-side batch ``step`` of this rank's contiguous shard (wraps around)."""
        n = len(self) // world
        start = rank * n + (step * batch_size) % max(1, n - batch_size + 1)
        return self.images[start:start + batch_size], self.labels[start:start + batch_size]


def mnist_splits(device="cpu", train: int = 60000, test: int = 10000, seed: int = 0):
    """(train, test) synthetic MNIST datasets sharing class templates."""
    full = SyntheticMNIST(train + test, device=device, seed=seed)
    tr, te = SyntheticMNIST.__new__(SyntheticMNIST), SyntheticMNIST.__new__(SyntheticMNIST)
    tr.images, tr.labels = full.images[:train], full.labels[:train]
    te.images, te.labels = full.images[train:], full.labels[train:]
    return tr, te


def resnet_batch(batch_size: int = 32, image: int = 128, classes: int = 1000, device="cpu", generator=None):
    """Random inputs + one-hot labels, as model_parallel_ResNet50.py:208-217."""
    x = torch.randn(batch_size, 3, image, image, generator=generator).to(device)
    idx = torch.randint(0, classes, (batch_size,), generator=generator)
    y = torch.zeros(batch_size, classes).scatter_(1, idx.view(batch_size, 1), 1).to(device)
    return x, y


def embbag_batches(rank: int = 0, num_batches: int = 10, num_embeddings: int = 100, classes: int = 8,
                   device="cpu", seed: int | None = None):
    """Yield (indices, offsets, targets) like server_model_data_parallel.py:49-68.

    20-50 indices in [0, num_embeddings); offsets with random gaps of 1-10 starting at 0; one target
    per bag in [0, classes).  The reference's ``get_next_batch(rank)`` call site passes a rank the
    function does not accept (TypeError, quirk Q1); here ``rank`` seeds the stream."""
    rng = random.Random(seed if seed is not None else 1234 + rank)
    for _ in range(num_batches):
        num_indices = rng.randint(20, 50)
        indices = torch.tensor([rng.randrange(num_embeddings) for _ in range(num_indices)], dtype=torch.long)
        offsets = []
        start = 0
        while start < num_indices:
            offsets.append(start)
            start += rng.randint(1, 10)
        offsets_t = torch.tensor(offsets, dtype=torch.long)
        targets = torch.tensor([rng.randrange(classes) for _ in offsets], dtype=torch.long)
        yield indices.to(device), offsets_t.to(device), targets.to(device)
