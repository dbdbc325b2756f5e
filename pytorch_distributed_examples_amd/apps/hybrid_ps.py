"""Hybrid parameter-server + data-parallel training (reference: rpc/server_model_data_parallel.py, R6),
and the ResNet-50 "2-stage pipeline x N-way DDP" hybrid of BASELINE config 4.

``--model embbag`` (default, the reference's workload): 4 processes -- 2 trainers, 1 master, 1 parameter
server ("ps").  The master builds ``RemoteModule("ps", EmbeddingBag(100, 16, mode="sum"))`` (:134-139)
and launches ``_run_trainer`` on both trainers (:142-152).  Each trainer's ``HybridModel`` = remote
embedding lookup + ``DDP(Linear(16, 8))`` (:34-46); 100 epochs over ``get_next_batch`` (the reference
calls it with an argument it does not accept -- TypeError, quirk Q1 fixed), distributed autograd, and a
``DistributedOptimizer(SGD, lr=0.05)`` over the remote table + local fc parameters (:78-105).  Each
trainer's step updates the PS table independently (Hogwild-style, Q16).  With GPUs the table lives in the
PS's HBM (EmbeddingBag gather / scatter-add HIP kernels) and the trainers' DDP runs on RCCL.

``--model resnet50 --stages 2 --dp 4`` (launch with torchrun, world = stages x dp): SPMD pipelines of
consecutive ranks (one xGMI link per stage pair), activations over RCCL P2P, and each stage's gradients
all-reduced across its data-parallel replicas (xGMI-sized buckets).
"""
from __future__ import annotations

import argparse
import os
import time

import torch
import torch.distributed as dist
import torch.distributed.rpc as rpc
import torch.multiprocessing as mp
from torch import nn, optim

from ..data.synthetic import embbag_batches
from ..ops import functional as OF
from ..ops import layers as L
from ..parallel.ddp import DistributedDataParallel
from ..parallel.dist import free_ports
from ..rpc import DistributedOptimizer, RemoteModule, dist_autograd
from ..utils import config as rtconfig
from ..utils.config import add_runtime_args

NUM_EMBEDDINGS = 100
EMBEDDING_DIM = 16


class HybridModel(nn.Module):
    """Remote EmbeddingBag on "ps" + DDP Linear(16, 8) local to the trainer (:34-46)."""

    def __init__(self, remote_emb_module, device, group):
        super().__init__()
        self.remote_emb_module = remote_emb_module
        self.fc = DistributedDataParallel(L.Linear(EMBEDDING_DIM, 8).to(device), process_group=group)
        self.device = device

    def forward(self, indices, offsets):
        # on GPUs the looked-up rows arrive in this GPU's HBM over the P2P ring (no host round trip)
        emb_lookup = self.remote_emb_module.forward(indices, offsets, out_device=self.device)
        return self.fc(emb_lookup.to(self.device), out_f32=True)


def get_next_batch(rank, num_batches=10, device="cpu"):
    yield from embbag_batches(rank=rank, num_batches=num_batches, num_embeddings=NUM_EMBEDDINGS, classes=8,
                              device=device)


def _run_trainer(remote_emb_module, rank, epochs, device_str):
    device = torch.device(device_str)
    model = HybridModel(remote_emb_module, device, dist.group.WORLD)
    model_parameter_rrefs = list(remote_emb_module.remote_parameters())
    for param in model.fc.parameters():
        model_parameter_rrefs.append(rpc.RRef(param))
    opt = DistributedOptimizer(optim.SGD, model_parameter_rrefs, lr=0.05)
    t0 = time.perf_counter()
    steps = 0
    for epoch in range(epochs):
        for indices, offsets, target in get_next_batch(rank):
            with dist_autograd.context() as context_id:
                output = model(indices, offsets)
                loss = OF.cross_entropy(output, target.to(device))
                dist_autograd.backward(context_id, [loss])
                opt.step(context_id)
            steps += 1
        if epoch % 5 == 0:
            print(f"Training done for epoch {epoch} (trainer {rank}, loss {loss.item():.4f})", flush=True)
    dt = time.perf_counter() - t0
    plane = "p2p-ring" if remote_emb_module.uses_ring(device) else "rpc-host"
    if remote_emb_module.uses_ring(device):
        remote_emb_module.close()
    print(f"trainer {rank}: {steps} steps, {dt / steps * 1e3:.2f} ms/step (embedding data plane: {plane})",
          flush=True)
    return steps


def run_worker(rank, world_size, epochs, ports, use_gpu):
    rpc_port, pg_port = ports
    options = rpc.TensorPipeRpcBackendOptions(num_worker_threads=16, rpc_timeout=300,
                                              init_method=f"tcp://127.0.0.1:{rpc_port}")
    ngpu = torch.cuda.device_count() if use_gpu else 0
    # the workload is a few KB per step: latency-bound.  One intra-op thread per process avoids 4 x 8
    # OpenMP teams spinning against each other on the host.
    torch.set_num_threads(1)
    if rank == 2:  # master
        rpc.init_rpc("master", rank=rank, world_size=world_size, rpc_backend_options=options)
        ps_dev = f"cuda:{2 % ngpu}" if use_gpu else "cpu"
        remote_emb_module = RemoteModule(f"ps/{ps_dev}", L.EmbeddingBag, args=(NUM_EMBEDDINGS, EMBEDDING_DIM),
                                         kwargs={"mode": "sum"})
        futs = []
        for trainer_rank in [0, 1]:
            dev = f"cuda:{trainer_rank % ngpu}" if use_gpu else "cpu"
            futs.append(rpc.rpc_async(f"trainer{trainer_rank}", _run_trainer,
                                      args=(remote_emb_module, trainer_rank, epochs, dev)))
        for fut in futs:
            fut.wait()
    elif rank <= 1:  # trainers: DDP group of 2 next to the RPC agent (:155-166)
        if use_gpu:
            torch.cuda.set_device(rank % ngpu)
        # PDE_BACKEND=gloo: trainers sharing one GPU (RCCL refuses two ranks on one device)
        dist.init_process_group(os.environ.get("PDE_BACKEND") or ("nccl" if use_gpu else "gloo"), rank=rank,
                                world_size=2, init_method=f"tcp://127.0.0.1:{pg_port}")
        rpc.init_rpc(f"trainer{rank}", rank=rank, world_size=world_size, rpc_backend_options=options)
    else:  # parameter server
        rpc.init_rpc("ps", rank=rank, world_size=world_size, rpc_backend_options=options)
    rpc.shutdown()
    if rank <= 1:
        dist.destroy_process_group()


# ------------------------------------------------------------------------------------------------
# ResNet-50 hybrid: pipeline stages x data parallel (SPMD under torchrun)
# ------------------------------------------------------------------------------------------------
class ResNetPipelineDP:
    """ResNet-50 in ``stages`` = 2 pipeline stages (one process / GPU each) x ``world / 2`` data-parallel
    replicas of every stage (SPMD: every rank builds the same object).

    * pipelines are consecutive ranks (0,1), (2,3), ...; stage ``s``'s replicas {s, s+2, ...} form the
      data-parallel group (``ncclCommSplit``-equivalent ``dist.new_group`` for control, and on GPUs a
      stream-ordered RCCL communicator of our own for the gradient all-reduce, so the whole step --
      micro-batch forwards/backwards, P2P sends/recvs, all-reduce, SGD -- records into ONE hipGraph);
    * ``split_size`` is the micro-batch size (reference quirk Q2), BatchNorm statistics are per micro-batch
      (Q17), each replica draws its own batch (seeded by pipeline index);
    * ``mb_group`` micro-batches form one pipeline unit, run as one launch sequence with grouped BatchNorm
      (per-micro-batch statistics, ``ops.functional.bn_groups``).  Default on the GPU: all of them (one unit
      per step -- at m = 4..32 the stage kernels are latency-bound, so one m = 32 pass beats four pipelined
      m = 8 passes: profiles/r3f_stage_bench.jsonl); ``PDE_PIPE_MB_GROUP`` / ``--mb-group`` override, 1 = the
      reference's one-micro-batch units;
    * ``step()`` runs one full training step and returns the loss on the last stage (a zero elsewhere).
    """

    def __init__(self, ctx, batch: int = 32, split_size: int = 8, image: int = 128, schedule: str = "gpipe",
                 lr: float = 0.05, tag: str = "hybrid", seed: int = 1234, mb_group: int | None = None):
        from ..data.synthetic import resnet_batch
        from ..models.resnet import ResNetShard1, ResNetShard2
        from ..ops.optim import FusedSGD
        from ..parallel.pipeline import PipelineEngine, hybrid_groups

        self.stages = 2
        world = ctx.world_size
        if world % self.stages:
            raise SystemExit(f"the ResNet-50 pipeline needs an even number of ranks (one per stage), got {world}")
        if batch % split_size:
            raise SystemExit(f"batch {batch} is not a multiple of the micro-batch size {split_size}")
        self.ctx = ctx
        self.dp = world // self.stages
        self.batch, self.split_size = batch, split_size
        _, dps = hybrid_groups(world, self.stages)
        self.stage = ctx.rank % self.stages
        self.last = self.stage == self.stages - 1
        groups = [dist.new_group(g) for g in dps]  # every rank creates every group (c10d requirement)
        self.dp_group = groups[self.stage]
        dev = ctx.device
        self.module = (ResNetShard1() if self.stage == 0 else ResNetShard2()).to(dev)
        self.comm = None
        # stage gradients: bf16 on the wire (our cast kernels around RCCL), reduced on a side stream during
        # the last micro-batch's backward (PDE_PIPE_DP_OVERLAP=0: one reduce after the pipeline drains)
        self.overlap = dev.type == "cuda" and self.dp > 1 and os.environ.get("PDE_PIPE_DP_OVERLAP", "1") != "0"
        dp_comm = os.environ.get("PDE_PIPE_DP_COMM", "rccl" if ctx.backend == "nccl" else "xgmi")
        if dev.type == "cuda" and self.dp > 1 and dp_comm == "rccl" and ctx.backend == "nccl":
            from ..parallel.rccl import StreamComm

            self.comm = StreamComm(dev, group=self.dp_group, side_stream=self.overlap)
        elif dev.type == "cuda" and self.dp > 1 and dp_comm == "gloo":
            self.overlap = False  # (diagnostic A/B: the c10d gloo group, host-staged; not capturable)
        elif dev.type == "cuda" and self.dp > 1:
            # the stage gradients over xGMI IPC (one-shot small, two-shot large buckets), no RCCL: the same code
            # runs with the 2 x dp ranks sharing ONE GPU (RCCL refuses duplicate devices), which is how the
            # config-4 step is rehearsed on a one-GPU box.  Reduced on the compute stream after the last
            # micro-batch's backward (the spinning exchange never competes with a one-launch BatchNorm for CUs).
            from ..parallel.xgmi_allreduce import xgmi_only_comm

            self.overlap = False
            self.comm = xgmi_only_comm(dev, group=self.dp_group, key=f"{tag}/dp{self.stage}")
        gd = torch.bfloat16 if (dev.type == "cuda" and os.environ.get("PDE_PIPE_GRAD_DTYPE", "bf16") == "bf16") else None
        self.ddp = DistributedDataParallel(self.module, process_group=self.dp_group,
                                           overlap=self.overlap and self.comm is not None,
                                           broadcast_buffers=False, comm=self.comm, grad_dtype=gd,
                                           static_graph=dev.type == "cuda")  # no zero fill (first writers store)
        self.opt = FusedSGD(self.module.parameters(), lr=lr)
        prev_rank = ctx.rank - 1 if self.stage > 0 else None
        next_rank = ctx.rank + 1 if not self.last else None
        self.engine = PipelineEngine(self.module, self.stage, self.stages, prev_rank, next_rank, dev,
                                     loss_fn=OF.mse_loss, schedule=schedule, tag=tag)
        if self.ddp.overlap:
            self.engine.ddp = self.ddp
        g = torch.Generator().manual_seed(seed + ctx.rank // self.stages)
        x, y = resnet_batch(batch, image, 1000, dev, g)
        n_mb = batch // split_size
        if mb_group is None:
            env = os.environ.get("PDE_PIPE_MB_GROUP")
            mb_group = int(env) if env else (n_mb if dev.type == "cuda" else 1)
        mb_group = max(1, min(int(mb_group), n_mb))
        while n_mb % mb_group:  # whole units only
            mb_group -= 1
        self.mb_group = mb_group
        self.engine.bn_groups = mb_group
        unit = split_size * mb_group
        self.n_mb = n_mb // mb_group  # pipeline units per step
        self.xs, self.ys = list(x.split(unit)), list(y.split(unit))
        self._zero = torch.zeros((), device=dev)

    @property
    def images_per_step(self) -> int:
        return self.batch * self.dp

    @property
    def capturable(self) -> bool:
        """The whole step can record into one hipGraph: GPU stage channels (ring / RCCL, not host staging)
        and a stream-ordered data-parallel communicator (or none at dp 1)."""
        if self.ctx.device.type != "cuda" or (self.dp > 1 and self.comm is None):
            return False
        return all(ch is None or ch.mode != "host" for ch in (self.engine.prev, self.engine.next))

    def check(self):
        """Raise if a stage channel or a one-launch BatchNorm hand-off timed out (synchronises the device)."""
        self.engine.check()

    def step(self, timer=None):
        """One training step; ``timer`` (utils.log.PhaseTimer, eager steps only): this stage's fwd / bwd /
        recv-wait / comm / opt device times."""
        from ..utils.log import NO_PHASES

        t = timer or NO_PHASES
        self.engine.timer = t
        self.ddp.zero_grad()
        loss = self.engine.train_step(self.xs if self.stage == 0 else None, self.ys if self.last else None,
                                      self.n_mb)
        with t.phase("comm"):
            if not self.ddp.overlap:  # (overlap: the hooks reduced every bucket during the last backward)
                self.ddp.sync_gradients()
        with t.phase("opt"):
            self.opt.step()
        self.engine.timer = NO_PHASES
        return loss if loss is not None else self._zero

    def split_step_graphs(self):
        """Ranks sharing ONE GPU (the config-4 rehearsal): the step as TWO hipGraphs -- the pipelined micro-batch
        forwards / backwards with their ring sends / receives, then the DP all-reduce + SGD -- with a device sync and
        a host barrier between them.  On a shared card a grid spinning on its DP peer starves the other pipeline's
        kernels (profiles/r6f), so no rank may start its DP exchange while another still computes; on a node (one
        GPU per rank) the step is ONE graph (``step``).  Runs ONE eager warm-up step in the same split form (ring
        meta handshake, lazy initialisation), then captures.  Returns a callable."""
        from ..utils.graph import CapturedStep

        def pipeline_part():
            self.ddp.zero_grad()
            loss = self.engine.train_step(self.xs if self.stage == 0 else None, self.ys if self.last else None,
                                          self.n_mb)
            return loss if loss is not None else self._zero

        def dp_part():
            self.ddp.sync_gradients()
            self.opt.step()
            return self._zero

        pipeline_part()  # the eager warm-up step, split the same way
        torch.cuda.synchronize()
        dist.barrier()
        dp_part()
        torch.cuda.synchronize()
        dist.barrier()
        g1 = CapturedStep(pipeline_part, [], warmup=0).capture()
        g2 = CapturedStep(dp_part, [], warmup=0).capture()

        def step():
            loss = g1()
            torch.cuda.synchronize()
            dist.barrier()
            g2()
            return loss

        return step

    def close(self):
        self.engine.close()
        if self.comm is not None:
            self.comm.destroy()


def run_resnet_hybrid(stages: int, dp: int, steps: int, warmup: int, batch: int, split_size: int,
                      schedule: str = "gpipe", quiet: bool = False, image: int = 128, device: str | None = None,
                      mb_group: int | None = None):
    from ..parallel import dist as pdist

    ctx = pdist.init_distributed(device=device)
    world = ctx.world_size
    assert world == stages * dp, f"world {world} != stages {stages} x dp {dp}"
    assert stages == 2, "ResNet-50 is split at layer2|layer3 (2 stages)"
    pipe = ResNetPipelineDP(ctx, batch, split_size, image, schedule, mb_group=mb_group)
    for _ in range(warmup):
        pipe.step()
    pdist.barrier(ctx)
    if ctx.device.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    loss = None
    for _ in range(steps):
        loss = pipe.step()
    pdist.barrier(ctx)
    if ctx.device.type == "cuda":
        torch.cuda.synchronize()
    pipe.check()  # ring waits and one-launch BatchNorm hand-offs of the run: raise on a timeout
    dt = pdist.max_over_ranks(time.perf_counter() - t0, ctx.device)
    img_s = pipe.images_per_step * steps / dt
    if not quiet and ctx.rank == stages - 1:
        print(f"resnet50 hybrid pp{stages} x dp{dp}: loss {loss.item():.4f} | {dt / steps * 1e3:.2f} ms/step | "
              f"{img_s:.1f} images/s (node)", flush=True)
    pipe.close()
    return pipe, img_s, dt / steps


def main(argv=None):
    ap = argparse.ArgumentParser(description="Hybrid PS + DDP (EmbeddingBag) / ResNet-50 pipeline x DDP")
    ap.add_argument("--model", default="embbag", choices=["embbag", "resnet50"])
    ap.add_argument("--epochs", type=int, default=100)
    ap.add_argument("--device", default="auto", choices=["auto", "cpu", "gpu"])
    ap.add_argument("--stages", type=int, default=2)
    ap.add_argument("--dp", type=int, default=None)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch-size", type=int, default=32)
    ap.add_argument("--split-size", type=int, default=8)
    ap.add_argument("--schedule", default="gpipe", choices=["gpipe", "1f1b"])
    ap.add_argument("--mb-group", type=int, default=None,
                    help="micro-batches per pipeline unit (grouped BatchNorm); default: all on the GPU")
    ap.add_argument("--image", type=int, default=128)
    add_runtime_args(ap)
    args = ap.parse_args(argv)
    _cfg = rtconfig.apply(rtconfig.from_args(args))
    if hasattr(args, "device"):
        args.device = rtconfig.device_for(_cfg, args.device)
    if args.model == "resnet50":
        world = int(os.environ.get("WORLD_SIZE", "1"))
        dp = args.dp or max(1, world // args.stages)
        run_resnet_hybrid(args.stages, dp, args.steps, args.warmup, args.batch_size, args.split_size,
                          args.schedule, image=args.image, device="cpu" if args.device == "cpu" else None,
                          mb_group=args.mb_group)
        dist.destroy_process_group()
        return
    use_gpu = torch.cuda.is_available() and args.device != "cpu"
    world_size = 4
    mp.spawn(run_worker, args=(world_size, args.epochs, tuple(free_ports(2)), use_gpu), nprocs=world_size,
             join=True)
