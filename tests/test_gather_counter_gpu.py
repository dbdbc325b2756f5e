"""Device-counter batch gather (csrc/kernels/elementwise.hip k_gather_rows_counter): the captured elastic step's
input node (elastic/rewire.py).  Against an index_select reference: eager launches advance the counter, a
hipGraph replayed k times gathers k consecutive slices, and a host rewrite of the counter repositions it."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_gather_rows_counter_matches_index_select(gpu):
    from pytorch_distributed_examples_amd import _native

    C = _native.C()
    g = torch.Generator().manual_seed(0)
    N, rows = 5000, 3 * 128
    images = torch.randn(N, 1, 28, 28, generator=g).to(gpu)
    labels = torch.randint(0, 10, (N,), generator=g).to(gpu)
    idx = torch.randperm(N, generator=g)[:4 * rows].to(gpu)
    counter = torch.zeros(2, dtype=torch.int32, device=gpu)
    x = torch.empty(rows, 1, 28, 28, device=gpu)
    y = torch.empty(rows, dtype=torch.long, device=gpu)

    def want(c):
        sl = idx[c * rows:(c + 1) * rows]
        return images.index_select(0, sl), labels.index_select(0, sl)

    for c in range(2):  # eager: the counter advances once per launch
        C.gather_rows_counter(images, labels, idx, counter, x, y)
        wx, wy = want(c)
        assert torch.equal(x, wx) and torch.equal(y, wy), c
    assert counter.tolist() == [2, 0]
    graph = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s), torch.cuda.graph(graph):
        C.gather_rows_counter(images, labels, idx, counter, x, y)
    torch.cuda.current_stream().wait_stream(s)
    counter.copy_(torch.tensor([1, 0], dtype=torch.int32))  # the host repositions (epoch start / resume)
    for c in (1, 2, 3):
        graph.replay()
        torch.cuda.synchronize()
        wx, wy = want(c)
        assert torch.equal(x, wx) and torch.equal(y, wy), c
    assert counter.tolist() == [4, 0]
