"""Horovod-style data-parallel MNIST CNN (reference: horovod/mnist_horovod.py).

Same structure as the reference: ``hvd.init()`` (:28), MNIST + ``DistributedSampler(num_replicas=
hvd.size(), rank=hvd.rank())`` with batch 1024 and no ``set_epoch`` (:34-44, quirk Q8 kept),
``SGD(lr=0.01)`` wrapped in ``hvd.DistributedOptimizer(named_parameters=...)`` (:50-53),
``hvd.broadcast_parameters(model.state_dict(), root_rank=0)`` (:56), 50 epochs of
zero_grad/forward/nll_loss/backward/step printing every 5 batches (:58-67).

MI355X-first: the model lives on this rank's GPU (the reference leaves ``torch.cuda.set_device`` and
``model.cuda()`` commented out, :31,:48); gradients are fused by the C++ engine and all-reduced with RCCL
over xGMI.  The GPU step (default; ``--layers`` keeps the layer-by-layer autograd path) is
:class:`..hvd.cnn_step.FusedHvdStep`: the whole-network fused kernel (csrc/kernels/cnn_fused.hip) writes the
gradients into one flat buffer, ``optimizer.step()`` = the engine's stream-ordered ``synchronize()`` (graph mode, one
xGMI exchange of the fused batch) + the multi-tensor SGD.  After one negotiated eager step the epoch runs as
hipGraph replays of ``--graph-chunk`` steps over this rank's shard gathered once (:mod:`..utils.epoch_graph`); the
every-5-batches loss lines are printed from pinned copies, without a sync in the loop.  A per-epoch
``images/s (node)`` line is added.
"""
from __future__ import annotations

import argparse
import time

import torch

from .. import hvd
from ..data.loader import ShardedLoader
from ..data.synthetic import mnist_splits
from ..models.cnn import Net
from ..ops import functional as OF
from ..ops.optim import FusedSGD
from ..parallel import dist as pdist
from ..utils.epoch_graph import AsyncLossLog
from ..utils import config as rtconfig
from ..utils.config import add_runtime_args


def main(argv=None):
    ap = argparse.ArgumentParser(description="Horovod-style MNIST CNN")
    ap.add_argument("--epochs", type=int, default=50)
    ap.add_argument("--batch-size", type=int, default=1024)
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--train-size", type=int, default=60000)
    ap.add_argument("--device", default="auto", choices=["auto", "cpu", "gpu"])
    ap.add_argument("--log-interval", type=int, default=5)
    ap.add_argument("--fused", action="store_true", help="fused whole-network training kernel (GPU; the default)")
    ap.add_argument("--layers", action="store_true", help="GPU: layer-by-layer autograd path instead")
    ap.add_argument("--graph-chunk", type=int, default=50, help="GPU: training steps per hipGraph replay")
    ap.add_argument("--compression", default="none", choices=["none", "fp16", "bf16"])
    add_runtime_args(ap)
    args = ap.parse_args(argv)
    _cfg = rtconfig.apply(rtconfig.from_args(args))
    if hasattr(args, "device"):
        args.device = rtconfig.device_for(_cfg, args.device)

    hvd.init(device="cpu" if args.device == "cpu" else None)
    dev = hvd.core._ctx.device
    train_set, _ = mnist_splits(device=dev, train=args.train_size, test=16)
    loader = ShardedLoader(train_set, args.batch_size, hvd.size(), hvd.rank(), shuffle=True)

    model = Net().to(dev)
    fast = dev.type == "cuda" and not args.layers
    optimizer = FusedSGD(model.parameters(), lr=args.lr)
    optimizer = hvd.DistributedOptimizer(optimizer, named_parameters=model.named_parameters(),
                                         compression=getattr(hvd.Compression, "bf16" if args.compression == "none"
                                                             and _cfg.grad_dtype == "bf16" else args.compression))
    step = runner = None
    if fast:
        from ..hvd.cnn_step import FusedHvdStep
        from ..utils.epoch_graph import ChunkedGraphs, EpochBatches

        # FusedHvdStep: its first call negotiates through the engine and turns graph mode on; the chunk graphs
        # then capture its eager body (fused kernel + synchronize + SGD) over the epoch buffer's slices
        step = FusedHvdStep(model, optimizer, args.batch_size, graph=False)
        eb = EpochBatches(loader)
        runner = ChunkedGraphs(step.eager_step, eb, chunk=args.graph_chunk, eager_first=1)
    hvd.broadcast_parameters(model.state_dict(), root_rank=0)

    def line(epoch):
        return lambda b, v: (f"Worker: {hvd.rank()} | Epoch: {epoch} | Batch: {b}/{len(loader)} | "
                             f"Loss: {v:.4f}")

    t0 = time.time()
    seen = 0
    for epoch in range(args.epochs):
        model.train()
        te = time.perf_counter()
        n = 0
        if runner is not None:
            eb.fill()  # no set_epoch, as in the reference (quirk Q8): the permutation repeats, so does no gather
            log = AsyncLossLog(line(epoch), args.log_interval)
            n, _ = runner.run(on_steps=log.add)
            eb.prepare(loader.sampler.epoch)  # the next epoch's (same, Q8) permutation while the GPU drains
            torch.cuda.synchronize()
            log.poll(wait=True)
        else:
            for batch_idx, (data, target) in enumerate(loader):
                optimizer.zero_grad()
                output = model(data)
                loss = OF.nll_loss(output, target)
                loss.backward()
                optimizer.step()
                n += data.shape[0]
                if batch_idx % args.log_interval == 0:
                    print(f"Worker: {hvd.rank()} | Epoch: {epoch} | Batch: {batch_idx}/{len(loader)} | "
                          f"Loss: {loss.item():.4f}", flush=True)
            if dev.type == "cuda":
                torch.cuda.synchronize()
        dt = time.perf_counter() - te
        seen += n
        node = pdist.sum_over_ranks(n / dt, torch.device("cpu"))
        if hvd.rank() == 0:
            print(f"Epoch {epoch} | train {dt:.3f}s | {node:.0f} images/s (node)", flush=True)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dt = time.time() - t0
    print(f"Worker: {hvd.rank()} | {seen / dt:.0f} images/s (this worker) | engine {hvd.engine_stats()}",
          flush=True)
    hvd.shutdown()
