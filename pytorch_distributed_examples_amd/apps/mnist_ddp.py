"""Elastic DDP MNIST trainer (reference: pytorch_elastic/mnist_ddp_elastic.py).

Launched by torchrun exactly like the reference (docstring at :1-7):

    torchrun --nnodes=1:2 --nproc_per_node=N --rdzv_backend=c10d --rdzv_endpoint=127.0.0.1:29603 \
        --max-restarts=3 pytorch_elastic/mnist_ddp_elastic.py 10 5 [--batch_size 128]

Behaviour kept from the reference: positional ``total_epochs save_every``, ``--batch_size`` (default 128;
the reference's help text says 32, :207), the MLP 5x1024 + Adam(1e-3) + CrossEntropy (:162-175), one
DistributedSampler shard per rank with ``set_epoch`` (:89), a per-rank test pass on the rank's test shard
after every epoch (:117-130; we also print the all-reduced global accuracy, Q6), snapshot every
``save_every`` epochs with the reference's keys and resume from it (Q4 semantics kept), the printed
lines, and ``Execution time``.

MI355X-first differences: RCCL (``nccl``) over xGMI on GPUs -- gloo on CPU -- with the xGMI bucket
policy; bf16 MFMA kernels; HBM-resident synthetic MNIST; atomic snapshot by global rank 0 only;
``--model cnn`` runs BASELINE config 1's CNN through the same plumbing; ``--rewire`` keeps the worker alive
across membership changes (in-process RCCL communicator re-wire, :mod:`..elastic.rewire`).

GPU training step (default; ``--layers`` keeps the layer-by-layer autograd + DDP-hook path of the CPU config):

* MLP, world 1: the whole step -- forward, cross-entropy, backward, Adam -- as ONE persistent launch
  (:class:`..models.mlp_mega.MegaMLP`); a short last batch whose size is not a multiple of 32 takes the layer path;
* MLP, world > 1: :class:`..models.mlp_fused.FusedMLP` (no autograd, dgrad + wgrad paired per layer) + the DDP flat
  buffer all-reduced by the stream-ordered RCCL / xGMI data plane + the multi-tensor Adam;
* CNN (``--fused`` is implied): the whole-network training kernel of csrc/kernels/cnn_fused.hip, gradients straight
  into the DDP flat buffer; on the xGMI data plane the all-reduce and the SGD update run inside its slab-reduction
  kernel, else one all-reduce and one fused SGD launch;
* the epoch runs as hipGraph replays of ``--graph_chunk`` steps each over this rank's shard gathered once per epoch
  (:mod:`..utils.epoch_graph`): no per-step host work.
"""
from __future__ import annotations

import argparse
import os
import time

import torch

from ..data.loader import ShardedLoader
from ..data.synthetic import mnist_splits
from ..elastic import fault
from ..elastic.snapshot import load_snapshot, save_snapshot
from ..ops import functional as OF
from ..ops.optim import FusedAdam, FusedSGD
from ..parallel import dist as pdist
from ..parallel.ddp import DistributedDataParallel
from ..utils.log import RankLogger, MetricsWriter
from ..utils import config as rtconfig
from ..utils.config import add_runtime_args


def load_train_objs(model_name: str, device, train_size: int, test_size: int):
    train_set, test_set = mnist_splits(device=device, train=train_size, test=test_size)
    if model_name == "cnn":
        from ..models.cnn import Net

        model = Net()
        loss = OF.nll_loss
        make_opt = lambda params: FusedSGD(params, lr=0.01)  # noqa: E731  (mnist_horovod.py:50)
    else:
        from ..models.mlp import reference_mlp

        model = reference_mlp()
        loss = OF.cross_entropy
        make_opt = lambda params: FusedAdam(params, lr=1e-3)  # noqa: E731  (mnist_ddp_elastic.py:173)
    return train_set, test_set, model, make_opt, loss


def _native_grid() -> int:
    from .. import _native

    return _native.C().mlp_train_grid()


class Trainer:
    def __init__(self, ctx, model, train_data, test_data, make_opt, criterion, save_every, snapshot_path,
                 log, metrics=None, save_optimizer=True, fused=False, ddp_kwargs=None, fast=None, graph_chunk=50):
        self.ctx = ctx
        self.global_rank = int(os.environ.get("RANK", ctx.rank))
        self.local_rank = int(os.environ.get("LOCAL_RANK", ctx.local_rank))
        self.model = model.to(ctx.device)
        self.train_data, self.test_data = train_data, test_data
        self.criterion = criterion
        self.save_every = save_every
        self.snapshot_path = snapshot_path
        self.epochs_run = 0
        self.log = log
        self.metrics = metrics
        self.save_optimizer = save_optimizer
        self.optimizer = make_opt(self.model.parameters())
        self.global_step = 0
        if os.path.exists(snapshot_path):
            log.print("Loading snapshot")
            self._load_snapshot(snapshot_path)
        self.fused = None
        self.fmlp = self.mega = None
        self.runner = None
        on_gpu = ctx.device.type == "cuda"
        is_cnn = type(self.model).__name__ == "Net"
        fast = on_gpu if fast is None else fast
        if fused and not on_gpu:
            raise SystemExit("--fused runs the gfx950 training kernel: it needs a GPU")
        if fast and not on_gpu:
            fast = False
        if (fused or fast) and is_cnn:
            from ..models.cnn_fused import FusedCNN
            from ..parallel.comm import data_plane

            self.fused = FusedCNN(self.model)
            # (the CNN's 87 KB of gradients is one one-shot bucket: no two-shot instance)
            self.ddp = DistributedDataParallel(self.model, overlap=False, param_order="forward",
                                               comm=data_plane(ctx, two_shot=False), **(ddp_kwargs or {}))
        elif fast:
            from ..models.mlp_fused import FusedMLP
            from ..parallel.comm import data_plane

            self.fmlp = FusedMLP(self.model)
            self.ddp = DistributedDataParallel(self.model, overlap=False, comm=data_plane(ctx), **(ddp_kwargs or {}))
            # one launch per step at any world size on one node: at world > 1 the gradient average runs inside the
            # launch over xGMI (MegaMLP.exchange) -- every rank must own its GPU (the persistent grid fills it)
            world = self.ddp.world
            own_gpu = torch.cuda.device_count() >= int(os.environ.get("LOCAL_WORLD_SIZE", "1"))
            single_node = int(os.environ.get("LOCAL_WORLD_SIZE", str(world))) == world
            if (train_data.batch_size % 32 == 0 and os.environ.get("PDE_MLP_MEGA", "1") != "0" and
                    (world == 1 or (own_gpu and single_node and getattr(self.optimizer, "KIND", "") != "sgd"))):
                from ..models.mlp_mega import MegaMLP

                if int(_native_grid()) > 0:
                    xa = MegaMLP.exchange(self.model, ctx.device) if world > 1 else None
                    self.mega = MegaMLP(self.model, self.optimizer, xgmi=xa)
        else:
            self.ddp = DistributedDataParallel(self.model, **(ddp_kwargs or {}))
        if (self.fused is not None or self.fmlp is not None) and hasattr(train_data.dataset, "images") and \
                os.environ.get("PDE_EPOCH_GRAPH", "1") != "0":
            from ..utils.epoch_graph import ChunkedGraphs, EpochBatches

            self.epoch_batches = EpochBatches(train_data)
            self.runner = ChunkedGraphs(self._gpu_step, self.epoch_batches, chunk=graph_chunk, eager_first=2,
                                        tail_step=self._gpu_tail_step)

    def _load_snapshot(self, path):
        snap = load_snapshot(path)
        self.model.load_state_dict(snap["MODEL_STATE"])
        if "OPTIMIZER_STATE" in snap:
            self.optimizer.load_state_dict(snap["OPTIMIZER_STATE"])
        self.epochs_run = snap["EPOCHS_RUN"]
        self.log.print(f"Resuming training from snapshot at Epoch {self.epochs_run}")

    def _gpu_step(self, source, targets):
        """One full-batch GPU training step (the function the epoch graphs capture)."""
        if self.mega is not None:
            return self.mega.step(source, targets)
        if self.fmlp is not None:
            loss = self.fmlp.forward_backward(source, targets)  # gradients written into the DDP flat buffer
            self.ddp.sync_gradients()
            self.optimizer.step()
            return loss
        return self._fused_cnn_step(source, targets)

    def _gpu_tail_step(self, source, targets):
        """The short last batch (eager): the one-launch MLP step needs a multiple of 32 rows."""
        if self.mega is not None and source.shape[0] % 32:
            loss = self.fmlp_for_tail().forward_backward(source, targets)
            self.ddp.sync_gradients()
            self.optimizer.step()
            return loss
        return self._gpu_step(source, targets)

    def fmlp_for_tail(self):
        if self.fmlp is None:
            from ..models.mlp_fused import FusedMLP

            self.fmlp = FusedMLP(self.model)
        return self.fmlp

    def _after_steps(self, idxs, losses):
        for _ in idxs:
            fault.maybe_fault(self.global_step, self.global_rank)
            self.global_step += 1

    def _fused_cnn_step(self, source, targets):
        xgmi = getattr(self.ddp.comm, "xgmi", None)
        if self.ddp.world == 1:  # SGD + fragment refresh inside the slab reduction
            return self.fused.forward_backward(source, targets, grad_out=self.ddp.flat_grad, sgd=self.optimizer)
        if xgmi is not None:  # + the gradient all-reduce, exchanged over xGMI inside that kernel
            return self.fused.forward_backward(source, targets, grad_out=self.ddp.flat_grad, sgd=self.optimizer,
                                               xgmi=xgmi)
        loss = self.fused.forward_backward(source, targets, grad_out=self.ddp.flat_grad)
        self.ddp.sync_gradients()
        self.fused.sgd_step(self.optimizer, self.ddp.flat_grad)
        return loss

    def _run_batch(self, source, targets):
        if self.fused is not None or self.fmlp is not None or self.mega is not None:
            loss = self._gpu_step(source, targets) if source.shape[0] == self.train_data.batch_size else \
                self._gpu_tail_step(source, targets)
            self._after_steps([0], [loss])
            return loss
        self.ddp.zero_grad()
        output = self.ddp(source)
        loss = self.criterion(output, targets)
        loss.backward()
        self.optimizer.step()
        fault.maybe_fault(self.global_step, self.global_rank)
        self.global_step += 1
        return loss

    def _run_epoch(self, epoch):
        self.model.train()
        b_sz = self.train_data.batch_size
        self.log.print(f"Local Rank: {self.local_rank} | Global Rank: {self.global_rank} | Epoch {epoch} | "
                       f"Batchsize: {b_sz} | Steps: {len(self.train_data)}", all_ranks=True)
        t0 = time.perf_counter()
        n = 0
        loss = None
        if self.runner is not None:  # hipGraph chunks over the epoch's gathered shard (utils/epoch_graph.py)
            self.epoch_batches.fill(epoch)
            n, loss = self.runner.run(on_steps=self._after_steps)
            self.epoch_batches.prepare(epoch + 1)  # host work while the GPU drains this epoch's replays
        else:
            self.train_data.set_epoch(epoch)
            for source, targets in self.train_data:
                loss = self._run_batch(source, targets)
                n += source.shape[0]
        if self.ctx.device.type == "cuda":
            torch.cuda.synchronize()
            if self.mega is not None:
                self.mega.check(f"rank {self.global_rank} epoch {epoch}")
            # a one-shot xGMI exchange that timed out drops its result (replicas would silently diverge):
            # read the device error word at this existing sync point, before the test pass and any snapshot
            check = getattr(self.ddp.comm, "check", None)
            if check is not None:
                check()
            OF.check_device_errors(f"rank {self.global_rank} epoch {epoch}")
        dt = time.perf_counter() - t0
        img_s = pdist.sum_over_ranks(n / dt, self.ctx.device)
        if self.metrics is not None:
            self.metrics.write(epoch=epoch, images_per_s=img_s, epoch_s=dt,
                               loss=float(loss.item()) if loss is not None else None)
        self.log.print(f"Epoch {epoch} | train {dt:.2f}s | {img_s:.0f} images/s (node)")
        self.test()

    def _save_snapshot(self, epoch):
        save_snapshot(self.snapshot_path, self.model.state_dict(), epoch,
                      self.optimizer.state_dict() if self.save_optimizer else None)
        self.log.print(f"Epoch {epoch} | Training snapshot saved at {self.snapshot_path}")

    def train(self, max_epochs: int):
        for epoch in range(self.epochs_run, max_epochs):
            self._run_epoch(epoch)
            if self.global_rank == 0 and epoch % self.save_every == 0:
                self._save_snapshot(epoch)

    @torch.no_grad()
    def test(self):
        # The reference never calls model.eval() (:117-130); we evaluate in eval mode (dropout off).
        was = self.model.training
        self.model.eval()
        correct = torch.zeros((), dtype=torch.long, device=self.ctx.device)
        total = 0
        for images, labels in self.test_data:
            outputs = self.model(images)
            predicted = outputs.float().argmax(1)
            total += labels.size(0)
            correct += (predicted == labels).sum()
        c = int(correct.item())
        self.log.print(f"Test accuracy: {(c / max(1, total)) * 100:.2f}%", all_ranks=True)
        gc = pdist.sum_over_ranks(c, self.ctx.device)
        gt = pdist.sum_over_ranks(total, self.ctx.device)
        self.log.print(f"Global test accuracy: {(gc / max(1, gt)) * 100:.2f}%")
        self.model.train(was)


def main(argv=None):
    parser = argparse.ArgumentParser(description="simple distributed training job")
    parser.add_argument("total_epochs", type=int, help="Total epochs to train the model")
    parser.add_argument("save_every", type=int, help="How often to save a snapshot")
    parser.add_argument("--batch_size", default=128, type=int, help="Input batch size on each device (default: 128)")
    parser.add_argument("--model", default="mlp", choices=["mlp", "cnn"])
    parser.add_argument("--fused", action="store_true",
                        help="cnn: whole-network fused training kernel (GPU; the default GPU path, kept for scripts)")
    parser.add_argument("--layers", action="store_true",
                        help="GPU: layer-by-layer autograd + DDP hooks instead of the fused / one-launch step")
    parser.add_argument("--graph_chunk", type=int, default=50, help="GPU: training steps per hipGraph replay")
    parser.add_argument("--device", default="auto", choices=["auto", "cpu", "gpu"])
    parser.add_argument("--snapshot_path", default="snapshot.pt")
    parser.add_argument("--train_size", type=int, default=60000)
    parser.add_argument("--test_size", type=int, default=10000)
    parser.add_argument("--metrics", default=None, help="JSONL metrics file (rank 0)")
    parser.add_argument("--rewire", action="store_true",
                        help="survive membership changes in-process (RCCL communicator re-wire); launch with "
                             "python -m pytorch_distributed_examples_amd.launch.hvdrun")
    parser.add_argument("--commit_every", type=int, default=10, help="--rewire: steps between in-memory commits")
    add_runtime_args(parser, style="underscore")
    args = parser.parse_args(argv)
    cfg = rtconfig.apply(rtconfig.from_args(args))
    args.device = rtconfig.device_for(cfg, args.device)

    start = time.time()
    if args.rewire and args.fused and args.model == "cnn":
        # the fused whole-step CNN with the gradient exchange over xGMI inside its reduction kernel, one hipGraph
        # per membership round (BASELINE config 2's data plane; CPU: the same protocol over autograd + gloo)
        from ..elastic.rewire import run_elastic_fused

        run_elastic_fused(args)
    elif args.rewire:
        from ..elastic.rewire import run_elastic

        run_elastic(args)
    else:
        ctx = pdist.init_distributed(device="cpu" if args.device == "cpu" else None)
        log = RankLogger(ctx.rank)
        metrics = MetricsWriter(args.metrics) if args.metrics and ctx.rank == 0 else None
        train_set, test_set, model, make_opt, criterion = load_train_objs(args.model, ctx.device, args.train_size,
                                                                          args.test_size)
        train_data = ShardedLoader(train_set, args.batch_size, ctx.world_size, ctx.rank, shuffle=True)
        test_data = ShardedLoader(test_set, args.batch_size, ctx.world_size, ctx.rank, shuffle=False)
        trainer = Trainer(ctx, model, train_data, test_data, make_opt, criterion, args.save_every,
                          args.snapshot_path, log, metrics, fused=args.fused and args.model == "cnn",
                          ddp_kwargs=cfg.ddp_kwargs(), fast=False if args.layers else None,
                          graph_chunk=args.graph_chunk)
        trainer.train(args.total_epochs)
        pdist.shutdown()
    end = time.time()
    print(f"Execution time: {end - start}")
