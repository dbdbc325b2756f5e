"""Horovod-elastic MNIST CNN (reference: horovod/horovod_mnist_elastic.py).

Kept from the reference: hyper-parameters ``epochs=15, batches_per_commit=30, lr=0.01`` (:12-14),
``AdamW(lr=0.01/sqrt(hvd.size()))`` + ``DistributedOptimizer`` (:41-42), ``get_dataset()`` re-sharding for
the current world inside ``train`` (:44-53,:58), ``@hvd.elastic.run`` with ``state.epoch``/``state.batch``
resume (:55-77), commit + print every 30 batches (:71-73), ``on_state_reset`` LR rescale (:80-82),
full-test-set accuracy on every rank at the end (:85-102), and ``TorchState(model, optimizer, batch=0,
epoch=0)`` + ``register_reset_callbacks`` (:104-106).

Launch (the reference's horovodrun line, :108):
    python -m pytorch_distributed_examples_amd.launch.hvdrun -np 2 --min-np 1 \
        --blacklist-cooldown-range 15 30 --host-discovery-script ./discover_hosts.sh \
        horovod_examples/horovod_mnist_elastic.py

Deliberate differences: skipped batches are not loaded (sampler offset, quirk Q10); the batch index
bookkeeping keeps the reference's "state.batch updated after the commit check" order.

On a GPU the step is :class:`..hvd.cnn_step.FusedHvdStep`: the fused whole-network CNN kernel, the fusion
engine's in-place all-reduce and the multi-tensor AdamW, captured into one hipGraph after the first (negotiated)
step and recaptured after every reset (``--no-graph``: eager; ``--layers``: the autograd layer path).
"""
from __future__ import annotations

import argparse
import math

import torch

from .. import hvd
from ..data.loader import ShardedLoader
from ..data.synthetic import mnist_splits
from ..elastic import fault
from ..models.cnn import Net
from ..ops import functional as OF
from ..ops.optim import FusedAdamW
from ..utils import config as rtconfig
from ..utils.config import add_runtime_args


def main(argv=None):
    ap = argparse.ArgumentParser(description="Horovod-elastic MNIST CNN")
    ap.add_argument("--epochs", type=int, default=15)
    ap.add_argument("--batches-per-commit", type=int, default=30)
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--batch-size", type=int, default=128)
    ap.add_argument("--train-size", type=int, default=60000)
    ap.add_argument("--test-size", type=int, default=10000)
    ap.add_argument("--device", default="auto", choices=["auto", "cpu", "gpu"])
    ap.add_argument("--layers", action="store_true", help="GPU: the autograd layer path instead of the fused step")
    ap.add_argument("--no-graph", action="store_true", help="GPU fused step without hipGraph capture")
    add_runtime_args(ap)
    args = ap.parse_args(argv)
    _cfg = rtconfig.apply(rtconfig.from_args(args))
    if hasattr(args, "device"):
        args.device = rtconfig.device_for(_cfg, args.device)
    epochs, batches_per_commit, lr = args.epochs, args.batches_per_commit, args.lr

    hvd.init(device="cpu" if args.device == "cpu" else None)
    dev = hvd.core._ctx.device
    train_set, test_set = mnist_splits(device=dev, train=args.train_size, test=args.test_size)

    model = Net().to(dev)
    optimizer = FusedAdamW(model.parameters(), lr=lr / math.sqrt(hvd.size()))
    optimizer = hvd.DistributedOptimizer(optimizer, named_parameters=model.named_parameters())
    step_counter = {"n": 0}
    fused_step = None
    if dev.type == "cuda" and not args.layers:
        from ..hvd.cnn_step import FusedHvdStep

        fused_step = FusedHvdStep(model, optimizer, args.batch_size, graph=not args.no_graph)

    def get_dataset():
        return ShardedLoader(train_set, args.batch_size, hvd.size(), hvd.rank(), shuffle=True)

    @hvd.elastic.run
    def train(state):
        print("Loading Dataset", flush=True)
        train_loader = get_dataset()
        print("Starting training", flush=True)
        batch_offset = state.batch
        for state.epoch in range(state.epoch, epochs):
            train_loader.start_batch = batch_offset
            for batch_idx, (data, target) in enumerate(train_loader, start=batch_offset):
                if fused_step is not None:
                    loss = fused_step(data, target)  # forward + backward + all-reduce + AdamW (one graph replay)
                else:
                    optimizer.zero_grad()
                    output = model(data)
                    loss = OF.nll_loss(output, target)
                    loss.backward()
                    optimizer.step()
                fault.maybe_fault(step_counter["n"], hvd.rank())
                step_counter["n"] += 1
                if state.batch % batches_per_commit == 0:
                    state.commit()
                    print(f"Worker: {hvd.rank()}/{hvd.size()} | Batch: {state.batch}/{len(train_loader)} | "
                          f"Epoch: {state.epoch} | Loss: {loss.item()}", flush=True)
                state.batch = batch_idx
            state.batch = 0
            batch_offset = 0

    def on_state_reset():
        for param_group in optimizer.param_groups:
            param_group["lr"] = lr / math.sqrt(hvd.size())
        if fused_step is not None:  # new engine / world / learning rate: renegotiate and recapture
            fused_step.reset()
        print(f"[elastic] reset: world {hvd.size()}, lr {lr / math.sqrt(hvd.size()):.6f}", flush=True)

    @torch.no_grad()
    def test():
        model.eval()
        loader = ShardedLoader(test_set, args.batch_size, 1, 0, shuffle=False)
        correct = total = 0
        for images, labels in loader:
            predicted = model(images).float().argmax(1)
            total += labels.size(0)
            correct += int((predicted == labels).sum().item())
        print(f"Accuracy: {(correct / total) * 100:.2f}%", flush=True)

    state = hvd.elastic.TorchState(model, optimizer, batch=0, epoch=0)
    state.register_reset_callbacks([on_state_reset])
    train(state)
    test()
    hvd.shutdown()
