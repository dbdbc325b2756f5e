"""The reference entry scripts on their default GPU paths: the one-launch MLP / fused CNN steps
replayed as hipGraph chunks over an epoch buffer (utils/epoch_graph.py), against the same steps run eagerly, and
the scripts' printed lines (pytorch_elastic/mnist_ddp_elastic.py:88,130,213; horovod/mnist_horovod.py:65-67)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _loader(n, B, gpu):
    from pytorch_distributed_examples_amd.data.loader import ShardedLoader
    from pytorch_distributed_examples_amd.data.synthetic import SyntheticMNIST

    ds = SyntheticMNIST(n, device=gpu, seed=3)
    return ShardedLoader(ds, B, 1, 0, shuffle=True)


def test_chunked_graphs_equal_eager_steps(gpu):
    """ChunkedGraphs (2 eager steps, then chunks of 3 steps, the short tail eager) == the same MegaMLP steps run
    one by one through the loader: same samples, same order, same weights and Adam state afterwards."""
    from pytorch_distributed_examples_amd.models.mlp import reference_mlp
    from pytorch_distributed_examples_amd.models.mlp_fused import FusedMLP
    from pytorch_distributed_examples_amd.models.mlp_mega import MegaMLP
    from pytorch_distributed_examples_amd.ops.optim import FusedAdam
    from pytorch_distributed_examples_amd.utils.epoch_graph import ChunkedGraphs, EpochBatches

    torch.manual_seed(0)
    ma = reference_mlp().to(gpu)
    mb = reference_mlp().to(gpu)  # (a deepcopy would drop the parameters' layer tags)
    mb.load_state_dict(ma.state_dict())
    oa, ob = FusedAdam(ma.parameters(), lr=1e-3), FusedAdam(mb.parameters(), lr=1e-3)
    mega_a, mega_b = MegaMLP(ma, oa), MegaMLP(mb, ob)
    fa, fb = FusedMLP(ma), FusedMLP(mb)

    def tail(f, o):
        def run(x, y):
            loss = f.forward_backward(x, y)
            o.step()
            return loss
        return run

    loader = _loader(128 * 11 + 40, 128, gpu)  # 11 full batches + a 40-row tail (not a multiple of 32)
    eb = EpochBatches(loader)
    runner = ChunkedGraphs(mega_b.step, eb, chunk=3, eager_first=2, tail_step=tail(fb, ob))
    for epoch in range(2):
        loader.set_epoch(epoch)
        la = []
        for x, y in loader:
            la.append((mega_a.step(x, y) if x.shape[0] == 128 else tail(fa, oa)(x, y)).item())
        eb.fill(epoch)
        lb = []
        runner.run(on_steps=lambda idxs, outs: lb.extend(o.item() for o in outs))
        assert len(lb) == len(la) == 12
        assert max(abs(a - b) for a, b in zip(la, lb)) < 1e-4, (la, lb)
    # epoch 0: 3 eager steps, chunks (3,3) (6,3) (9,2), eager tail; epoch 1: chunk (0,3) captured too
    assert runner.captures == 4 and runner.replays == 7
    for pa, pb in zip(ma.parameters(), mb.parameters()):
        torch.testing.assert_close(pa, pb, rtol=1e-4, atol=1e-5)
    assert mega_a.errors() == 0 and mega_b.errors() == 0


def test_mnist_ddp_entry_default_gpu_path(gpu, tmp_path, capsys):
    """pytorch_elastic/mnist_ddp_elastic.py's default (MLP, world 1) on the GPU: the one-launch step in epoch
    graphs; the reference's lines, a snapshot with its keys, and training progress."""
    from pytorch_distributed_examples_amd.apps import mnist_ddp

    snap = tmp_path / "snapshot.pt"
    mnist_ddp.main(["2", "1", "--train_size", "6400", "--test_size", "1024", "--snapshot_path", str(snap),
                    "--metrics", str(tmp_path / "m.jsonl")])
    out = capsys.readouterr().out
    assert "Batchsize: 128 | Steps: 50" in out and "images/s (node)" in out and "Test accuracy" in out
    assert "Execution time" in out and snap.exists()
    import json

    rows = [json.loads(l) for l in open(tmp_path / "m.jsonl")]
    assert len(rows) == 2 and rows[1]["loss"] < rows[0]["loss"] + 0.5
    sd = torch.load(snap, weights_only=True)
    assert {"MODEL_STATE", "EPOCHS_RUN"} <= set(sd)


def test_mnist_hvd_entry_default_gpu_path(gpu, capsys):
    """horovod/mnist_horovod.py's GPU default: FusedHvdStep (fused kernel + engine synchronize + SGD) in epoch
    graphs; the every-5-batches loss lines come out in order without a sync in the loop."""
    from pytorch_distributed_examples_amd.apps import mnist_hvd

    mnist_hvd.main(["--epochs", "2", "--train-size", "16384", "--log-interval", "5", "--graph-chunk", "4"])
    out = capsys.readouterr().out
    lines = [l for l in out.splitlines() if l.startswith("Worker: 0 | Epoch: 1 | Batch:")]
    assert [int(l.split("Batch: ")[1].split("/")[0]) for l in lines] == [0, 5, 10, 15]
    losses = [float(l.rsplit("Loss: ", 1)[1]) for l in lines]
    assert all(0.0 < v < 5.0 for v in losses)
    assert "images/s (node)" in out and "images/s (this worker)" in out
