"""utils/epoch_graph.py on the CPU: the tensor form of DistributedSampler's indices, the epoch buffer's batches
against ShardedLoader's, and the chunk runner's eager fallback (no GPU: every step eager, same order)."""
import pytest
import torch
from torch.utils.data.distributed import DistributedSampler


class _DS:
    def __init__(self, n):
        self.images = torch.arange(n * 4, dtype=torch.float32).view(n, 4)
        self.labels = torch.arange(n)

    def __len__(self):
        return self.labels.numel()


@pytest.mark.parametrize("n,world,shuffle,drop", [(100, 1, True, False), (103, 4, True, False), (5, 8, True, False),
                                                   (103, 3, False, False), (103, 4, True, True)])
def test_sampler_indices_match_distributed_sampler(n, world, shuffle, drop):
    from pytorch_distributed_examples_amd.utils.epoch_graph import sampler_indices

    for rank in range(world):
        s = DistributedSampler(_DS(n), num_replicas=world, rank=rank, shuffle=shuffle, seed=7, drop_last=drop)
        for epoch in (0, 3):
            s.set_epoch(epoch)
            assert sampler_indices(s).tolist() == list(iter(s))


def test_epoch_batches_and_runner_follow_the_loader():
    from pytorch_distributed_examples_amd.data.loader import ShardedLoader
    from pytorch_distributed_examples_amd.utils.epoch_graph import AsyncLossLog, ChunkedGraphs, EpochBatches

    ds = _DS(70)
    loader = ShardedLoader(ds, 8, num_replicas=2, rank=1, shuffle=True)
    eb = EpochBatches(loader)
    seen = []
    runner = ChunkedGraphs(lambda x, y: (seen.append(y.clone()), x.sum())[1], eb, chunk=3)
    assert not runner.enabled  # no GPU: every step eager
    lines = []
    log = AsyncLossLog(lambda b, v: f"{b}:{v:.0f}", every=2)
    import builtins

    orig = builtins.print
    builtins.print = lambda *a, **k: lines.append(a[0])
    try:
        for epoch in (0, 1):
            loader.set_epoch(epoch)
            want = [y for _, y in loader]
            eb.fill(epoch)
            seen.clear()
            n, _ = runner.run(on_steps=log.add)
            log.poll(wait=True)
            assert n == 35 and len(seen) == len(want) == 5
            assert all(torch.equal(a, b) for a, b in zip(seen, want))
    finally:
        builtins.print = orig
    assert [l.split(":")[0] for l in lines] == ["0", "2", "4", "0", "2", "4"]
