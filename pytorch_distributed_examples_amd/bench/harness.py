"""Images/sec benchmark harness behind the root ``bench.py`` (BASELINE.json metric).

Workloads (``--model``), one process per GPU, synthetic data resident in HBM, random init:

* ``cnn`` (default) -- BASELINE config 1: the reference's MNIST CNN ``Net`` (horovod/mnist_horovod.py:9-25)
  at its per-worker batch 1024 (:44), SGD lr 0.01 (:50), NLL on log_softmax; data parallel over RCCL.  The
  whole forward+loss+backward runs in one fused kernel (csrc/kernels/cnn_fused.hip).
* ``mlp`` -- the elastic-DDP script's 5x1024 MLP (pytorch_elastic/mnist_ddp_elastic.py:133-173), batch 128,
  Adam 1e-3, cross-entropy; data parallel.
* ``resnet50`` -- ResNet-50 at 128x128, batch 32, MSE, SGD 0.05, pure data parallel.
* ``resnet50_stage`` -- ONE pipeline stage of configs 3/4 at micro-batch size ``--batch`` (default 8, the
  reference's split size): ``--stage 1`` = stem+layer1+layer2 on images, ``--stage 2`` = layer3+layer4+fc on a
  [m,16,16,512] bf16 activation with MSE; each step is forward, backward against an upstream gradient
  (stage 1) / the loss (stage 2, input gradient included: it goes upstream), SGD -- what one stage GPU does
  per micro-batch, minus the P2P transfers.
* ``hvd_cnn`` -- BASELINE config 1's CNN through the HOROVOD path (horovod/mnist_horovod.py:47-67):
  ``hvd.DistributedOptimizer(FusedSGD)`` + ``hvd.broadcast_parameters``; the first step negotiates every
  gradient through the C++ fusion engine (filling its response cache), then the optimizer switches to graph
  mode (the cached batches enqueued stream-ordered: one in-place one-shot xGMI all-reduce of the fused
  model's flat gradient buffer) and the whole step records into a hipGraph.  World 1: Horovod's all-reduce is
  the identity, so the step is the fused kernel with the SGD update in its reduction (2 launches).
* ``hvd_cnn_elastic`` -- the Horovod-ELASTIC script's step (horovod/horovod_mnist_elastic.py:41-52): batch 128,
  ``hvd.DistributedOptimizer(AdamW(lr=0.01/sqrt(size)))``; the fused kernel's gradients (weight fragments rebuilt
  in-kernel every step: the optimiser is not the fused SGD), the engine's in-place all-reduce in graph mode and
  the multi-tensor AdamW, recorded into hipGraphs (:class:`..hvd.cnn_step.FusedHvdStep` is the same step in the
  elastic script itself).
* ``resnet50_pp`` -- BASELINE configs 3 and 4: the 2-stage ResNet-50 of rpc/model_parallel_ResNet50.py
  (stem+layer1+layer2 | layer3+layer4+fc, :85-139), batch 32 split into micro-batches of ``--split-size``
  (the reference's ``split_size`` semantics, :171, quirk Q2), one stage per GPU, activations and their
  gradients GPU->GPU over RCCL P2P (one direct xGMI link per stage pair), and ``world/2``-way data parallel
  over each stage's replicas (world 2 = config 3, world 8 = pp2 x dp4 = config 4).

Every timed step is a complete training step (forward, backward, gradient all-reduce, optimizer update);
steps are recorded into hipGraphs (several steps per replay for the launch-bound MNIST nets).  W warmup steps
run untimed; then K steps are timed between barrier + synchronize pairs and the MAX over ranks is taken.

Multi-GPU runs verify themselves: the world size must equal ``--gpus``, and every rank all-reduces a
checksum over the GPU data-plane communicator and reads back RCCL's own rank count (``rccl_nranks``).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

from ..parallel import dist as pdist
from ..utils.log import NO_PHASES, PhaseTimer

# BASELINE.json names one metric for the whole suite; ``config`` says which of its workloads this run measured.
METRIC = "images/sec (whole node) MNIST DDP + ResNet50 RPC-MP at 1/2/4/8 MI355X"
BASELINE_CONFIG = {"cnn": "1: MNIST CNN DDP bf16, RCCL allreduce over xGMI",
                   "hvd_cnn": "1 via the Horovod API (horovod/mnist_horovod.py DistributedOptimizer)",
                   "hvd_cnn_elastic": "the Horovod-elastic script's step (horovod_mnist_elastic.py: AdamW, batch 128)",
                   "mlp": "0/1 workload of mnist_ddp_elastic.py (5x1024 MLP DDP)",
                   "resnet50": "ResNet-50 128px data parallel (no BASELINE config; kernel reference point)",
                   "resnet50_stage": "one stage of configs 3/4 at micro-batch size (per-stage kernel time)",
                   "resnet50_pp": "3 (world 2: ResNet50 model-parallel across 2 MI355X) / "
                                  "4 (world 8: 2-stage pipeline x 4-way DDP)"}
# The reference's own numbers, measured on CPU by the survey (no published figures exist).
# Only same-workload, same-world comparisons are reported.
REFERENCE_IMG_S = {("mlp", 1): 7452.0, ("mlp", 2): 2630.0, ("mlp", 4): 4620.0,
                   ("resnet50_pp", 2): 18.0}
DEFAULT_BATCH = {"cnn": 1024, "hvd_cnn": 1024, "hvd_cnn_elastic": 128, "mlp": 128, "resnet50": 32, "resnet50_stage": 8, "resnet50_pp": 32}
MODEL_NAMES = {"cnn": "mnist_cnn_Net", "hvd_cnn": "mnist_cnn_Net", "hvd_cnn_elastic": "mnist_cnn_Net", "mlp": "mnist_mlp_5x1024", "resnet50": "resnet50_128px",
               "resnet50_stage": "resnet50_128px_stage", "resnet50_pp": "resnet50_128px_2stage"}


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); bench.py launches them when run without torchrun")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--model", default="cnn",
                    choices=["cnn", "hvd_cnn", "hvd_cnn_elastic", "mlp", "resnet50", "resnet50_stage", "resnet50_pp",
                             "resnet50_hybrid", "elastic_cnn"])
    ap.add_argument("--stage", type=int, default=1, choices=[1, 2], help="resnet50_stage: which pipeline stage")
    ap.add_argument("--scale-to", type=int, default=None, help="elastic_cnn: world size after the first round")
    ap.add_argument("--fault-at", type=int, default=None,
                    help="elastic_cnn: the last rank exits at this training step; the survivors re-wire in-process")
    ap.add_argument("--elastic-worker", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--hosts-file", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--report", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--batch", type=int, default=None, help="per-replica batch")
    ap.add_argument("--split-size", type=int, default=8, help="resnet50_pp: micro-batch size (reference: 4 or 8)")
    ap.add_argument("--schedule", default="gpipe", choices=["gpipe", "1f1b"], help="resnet50_pp schedule")
    ap.add_argument("--mb-group", type=int, default=None,
                    help="resnet50_pp: micro-batches per pipeline unit, run as one launch sequence with grouped "
                         "(per-micro-batch) BatchNorm; default: all of them on the GPU (PDE_PIPE_MB_GROUP)")
    ap.add_argument("--image", type=int, default=None, help="override the image size (CPU plumbing tests)")
    ap.add_argument("--no-graph", action="store_true", help="run the step eagerly (no hipGraph capture)")
    ap.add_argument("--graph-steps", type=int, default=0,
                    help="consecutive training steps recorded into one hipGraph (each reads its own batch); "
                         "0 = auto: the largest divisor of --steps up to 50 -- and up to --warmup when that still "
                         "leaves >= 4 steps per graph -- so the timed steps are whole replays of a graph the warmup "
                         "already replayed")
    ap.add_argument("--generic", action="store_true", help="CNN / MLP: layer-by-layer autograd kernels instead of the fused step")
    ap.add_argument("--device", default="auto", choices=["auto", "cpu"], help="cpu: contract/plumbing check only")
    args = ap.parse_args(argv)
    if args.graph_steps <= 0:
        def divisor_upto(cap):
            return max(d for d in range(1, max(1, min(cap, args.steps)) + 1) if args.steps % d == 0)
        # a group the warmup replays at least once: the FIRST replay of a freshly captured multi-step graph ran
        # ~0.1 ms slow in half of the processes (driver config, 20 / 5: 0.0325 vs 0.0286 ms/step when the 20-step
        # graph was first replayed inside the timed region, 0.0285-0.0288 with a 5-step graph the warmup had
        # replayed; profiles/README.md r6ae)
        g = divisor_upto(min(50, args.warmup))
        args.graph_steps = g if g >= 4 else divisor_upto(50)
    if args.model == "resnet50_hybrid":
        args.model = "resnet50_pp"
    return args


class Workload:
    """What the timing loop needs: a step callable, an optional multi-step graph, the images per step."""

    def __init__(self, step, images_per_step, parallelism, **info):
        self.step = step              # step(i) -> loss (device tensor or None)
        self.group = None             # CapturedSteps running several steps per replay
        self.images_per_step = images_per_step
        self.parallelism = parallelism
        self.info = info
        self.loss_rank = 0            # the rank whose loss is reported


def _data_plane_check(ctx, comm) -> int:
    """Checksum all-reduce over the data-plane communicator; returns the rank count it reports."""
    n = ctx.world_size
    if n == 1:
        return 1
    want = n * (n + 1) / 2
    t = torch.full((16,), float(ctx.rank + 1), device=ctx.device)
    if comm is not None:
        comm.allreduce_(t)
        nranks = comm.rccl.nranks()
    else:
        dist.all_reduce(t)
        nranks = dist.get_world_size()
    if not bool((t == want).all()):
        raise RuntimeError(f"rank {ctx.rank}: data-plane checksum {t[0].item()} != {want}")
    if nranks != n:
        raise RuntimeError(f"rank {ctx.rank}: communicator reports {nranks} ranks, world is {n}")
    return nranks


_UNIT_GRADS: dict = {}


def _unit_grad(loss):
    """A persistent d loss / d loss = 1 (``loss.backward()`` fills a fresh one every step: an ATen fill kernel)."""
    key = (loss.dtype, loss.device, tuple(loss.shape))
    if key not in _UNIT_GRADS:
        _UNIT_GRADS[key] = torch.ones_like(loss)
    return _UNIT_GRADS[key]


def _capture(step_fn, batches, graph_steps, rank):
    """(single-step graph, multi-step graph) or (None, None) when capture is not possible."""
    from ..utils.graph import CapturedStep, CapturedSteps

    try:
        one = CapturedStep(step_fn, batches[0], warmup=3).capture()
        group = None
        if graph_steps > 1:
            group = CapturedSteps(step_fn, [batches[j % len(batches)] for j in range(graph_steps)], warmup=1).capture()
        return one, group
    except Exception as exc:  # capture unsupported (e.g. a collective that cannot be captured): run eagerly
        if rank == 0:
            print(f"[bench] hipGraph capture failed, running eagerly: {exc}", file=sys.stderr)
        from .. import _native

        torch.cuda.synchronize()
        _native.C().clear_last_error()  # the aborted capture leaves a sticky "last error" behind
        return None, None


def build_data_parallel(args, ctx, batch) -> Workload:
    from ..ops import functional as OF
    from ..ops.optim import FusedAdam, FusedSGD
    from ..parallel.ddp import DistributedDataParallel

    dev = ctx.device
    on_gpu = dev.type == "cuda"
    torch.manual_seed(0)  # reproducible random init (the same weights on every rank before the broadcast)
    if args.model in ("cnn", "mlp"):
        from ..data.synthetic import SyntheticMNIST

        data = SyntheticMNIST(max(8 * batch, 16384), device=dev, seed=0)

        def batch_fn(i):
            return data.batch(i, batch)

        if args.model == "cnn":
            from ..models.cnn import Net

            model = Net().to(dev)
            opt = FusedSGD(model.parameters(), lr=0.01)
            loss_fn = OF.nll_loss
        else:
            from ..models.mlp import reference_mlp

            model = reference_mlp().to(dev)
            opt = FusedAdam(model.parameters(), lr=1e-3)
            loss_fn = OF.cross_entropy
    elif args.model == "resnet50_stage":
        from ..data.synthetic import resnet_batch
        from ..models.resnet import ResNetShard1, ResNetShard2

        img = args.image or 128
        g = torch.Generator().manual_seed(0)
        model = (ResNetShard1() if args.stage == 1 else ResNetShard2()).to(dev)
        opt = FusedSGD(model.parameters(), lr=0.05)
        if args.stage == 1:
            x, _ = resnet_batch(batch, img, 1000, dev, g)
            with torch.no_grad():
                yshape = model(x).shape
            # the gradient stage 2 would send back for the stage-1 output (train_step: out.backward(dy))
            dy = (torch.randn(yshape, generator=g) * 1e-3).to(dev, model(x).dtype)
            loss_fn = None
            batches = [(x, dy)]
        else:
            s1 = ResNetShard1().to(dev)
            x0, y = resnet_batch(batch, img, 1000, dev, g)
            with torch.no_grad():
                act = s1(x0)  # a stage-1 activation of the native layout (NHWC bf16 on GPU)
            del s1
            loss_fn = OF.mse_loss
            batches = [(act.requires_grad_(True), y)]  # its gradient goes upstream: dgrad of layer3's first convs

        def batch_fn(i):
            return batches[0]
    else:
        from ..data.synthetic import resnet_batch
        from ..models.resnet import ResNet50

        model = ResNet50().to(dev)
        g = torch.Generator().manual_seed(0)
        batches = [resnet_batch(batch, args.image or 128, 1000, dev, g) for _ in range(2)]
        opt = FusedSGD(model.parameters(), lr=0.05)
        loss_fn = OF.mse_loss

        def batch_fn(i):
            return batches[i % 2]

    # resnet50_stage --mb-group G: the stage's batch is G micro-batches run as one unit (grouped BatchNorm)
    bn_groups = (args.mb_group or 1) if args.model == "resnet50_stage" else 1
    if batch % bn_groups:
        raise SystemExit(f"--batch {batch} is not a multiple of --mb-group {bn_groups}")
    use_graph = not args.no_graph and on_gpu and (ctx.world_size == 1 or ctx.backend == "nccl")
    # GPU data plane for world > 1: our stream-ordered RCCL communicator (c10d's ProcessGroupNCCL aborts the
    # process when its work is captured into a hipGraph on ROCm -- parallel/rccl.py)
    # GPU data plane (parallel/comm.py): RCCL + the one-shot xGMI all-reduce for latency-bound buckets (the
    # CNN's single 87 KB bucket)
    from ..parallel.comm import data_plane

    comm = data_plane(ctx, two_shot=args.model.startswith("resnet50"))  # (the MNIST nets' buckets are one-shot sized)
    nranks = _data_plane_check(ctx, getattr(comm, "rccl", comm))
    fused = None
    if args.model == "cnn" and not args.generic and on_gpu:
        # whole-network fused kernel: gradients land in the DDP flat buffer (forward layout), then one
        # all-reduce and one fused SGD launch that also refreshes the kernel's bf16 weight fragments
        # (world 1: the SGD runs inside the slab reduction)
        from ..models.cnn_fused import FusedCNN

        fused = FusedCNN(model)
        fmlp = None
        ddp = DistributedDataParallel(model, overlap=False, param_order="forward", comm=comm)
    else:
        fmlp = None
        if args.model == "mlp" and not args.generic and on_gpu:
            # explicit launch sequence, no autograd: weight + bias gradients of each layer in ONE GEMM
            from ..models.mlp_fused import FusedMLP

            fmlp = FusedMLP(model)
        # ResNet-50 / stages: every gradient's first writer stores (conv / linear weight gradients, BatchNorm's
        # finalize), so after two checked steps zero_grad stops filling the 100 MB flat gradient
        ddp = DistributedDataParallel(model, overlap=not use_graph and fmlp is None, comm=comm,
                                      static_graph=on_gpu and args.model.startswith("resnet50"))
    # world 1, fused MLP, PDE_MLP_FOLD_OPT=1: each layer's Adam update appended to the next backward GEMM launch
    # (default: the separate multi-tensor launch after backward -- measured faster, profiles/README.md r3k)
    fold_opt = fmlp is not None and ctx.world_size == 1 and os.environ.get("PDE_MLP_FOLD_OPT", "0") == "1"
    # fused MLP: the whole step (forward, loss, backward, Adam) as ONE persistent launch (models/mlp_mega.py;
    # PDE_MLP_MEGA=0: the layer-by-layer launches) -- at world > 1 on one node with a GPU per rank the gradient
    # average runs inside that launch over xGMI (MegaMLP.exchange), as in the entry script (apps/mnist_ddp.py)
    mega = None
    mega_xchg = False
    if fmlp is not None and not fold_opt and os.environ.get("PDE_MLP_MEGA", "1") != "0" and batch % 32 == 0:
        local = int(os.environ.get("LOCAL_WORLD_SIZE", str(ctx.world_size)))
        own_gpu = torch.cuda.device_count() >= local
        mega_xchg = (ctx.world_size > 1 and own_gpu and local == ctx.world_size and
                     getattr(opt, "KIND", "") != "sgd" and os.environ.get("PDE_MLP_MEGA_XCHG", "1") != "0")
        if ctx.world_size == 1 or mega_xchg:
            from ..models.mlp_mega import MegaMLP

            if int(OF._C().mlp_train_grid()) > 0:
                xa = MegaMLP.exchange(model, ctx.device) if ctx.world_size > 1 else None
                mega = MegaMLP(model, opt, xgmi=xa)
        mega_xchg = mega_xchg and mega is not None
    # world > 1 on the xGMI data plane: the fused CNN exchanges its gradients inside the slab reduction
    # (PDE_CNN_XCHG=0: all-reduce through the DDP communicator + a separate SGD launch instead)
    xgmi = getattr(comm, "xgmi", None) if fused is not None and os.environ.get("PDE_CNN_XCHG", "1") != "0" else None

    def train_step(x, y, t=NO_PHASES):
        # ``t``: PhaseTimer of the phase measurement (eager steps after the timed region), else a no-op
        if fused is not None:
            if ctx.world_size == 1:
                with t.phase("fused_fwd_bwd_reduce_sgd"):
                    return fused.forward_backward(x, y, grad_out=ddp.flat_grad, sgd=opt)
            if xgmi is not None:  # all-reduce folded into the slab reduction: still 2 launches per step
                with t.phase("fused_fwd_bwd_xchg_sgd"):
                    return fused.forward_backward(x, y, grad_out=ddp.flat_grad, sgd=opt, xgmi=xgmi)
            with t.phase("fused_fwd_bwd_reduce"):
                loss = fused.forward_backward(x, y, grad_out=ddp.flat_grad)
            with t.phase("comm"):
                ddp.sync_gradients()
            with t.phase("opt"):
                fused.sgd_step(opt, ddp.flat_grad)
            return loss
        if mega is not None:
            with t.phase("mega_fwd_loss_bwd_adam"):
                return mega.step(x, y)
        if fmlp is not None:
            if fold_opt:  # one process: the optimiser step rides on the backward launches (FusedMLP)
                with t.phase("fwd_bwd_opt"):
                    return fmlp.forward_backward(x, y, opt=opt)
            with t.phase("fwd_bwd"):
                loss = fmlp.forward_backward(x, y)  # gradients written (not accumulated): no zeroing
            if ctx.world_size > 1:
                with t.phase("comm"):
                    ddp.sync_gradients()
            with t.phase("opt"):
                opt.step()
            return loss
        ddp.zero_grad()
        if x.requires_grad:
            x.grad = None  # a stage input: its gradient is produced fresh every step (sent upstream)
        if loss_fn is None:  # a pipeline stage without the loss: backward from the upstream gradient y
            with t.phase("fwd"), OF.bn_groups(bn_groups):
                out = ddp(x)
            with t.phase("bwd"):
                out.backward(y)
            loss = None
        else:
            with t.phase("fwd"), OF.bn_groups(bn_groups):
                loss = loss_fn(ddp(x), y)
            with t.phase("bwd"):
                loss.backward(_unit_grad(loss))
        if not ddp.overlap:  # graph mode: buckets reduced after backward on the capturing stream
            with t.phase("comm"):
                ddp.sync_gradients()
        with t.phase("opt"):
            opt.step()
        return loss

    one = group = None
    if use_graph:
        one, group = _capture(train_step, [batch_fn(j) for j in range(max(1, args.graph_steps))],
                              args.graph_steps, ctx.rank)
        if one is None and fused is None and fmlp is None:  # eager fallback: overlapped buckets (hooks) again
            ddp.remove_hooks()
            ddp = DistributedDataParallel(model, overlap=True, comm=comm)

    def step(i):
        x, y = batch_fn(i)
        return one(x, y) if one is not None else train_step(x, y)

    routed = getattr(comm, "routed", None)
    extra = {"stage": args.stage, "mb_per_unit": bn_groups} if args.model == "resnet50_stage" else {}
    w = Workload(step, batch * ctx.world_size, f"dp{ctx.world_size}", **extra, hipgraph=one is not None,
                 fused_step=fused is not None or fmlp is not None, rccl_nranks=nranks,
                 **({"optimizer": "adam folded into the backward launches"} if fold_opt else {}),
                 **({"mega_kernel": True, "launches_per_step": mega.kernel_launches_per_step(),
                     "optimizer": "adam inside the step's single launch"} if mega is not None else {}),
                 steps_per_graph=group.steps if group is not None else (1 if one is not None else 0),
                 allreduce=("xgmi-in-mega-kernel" if mega_xchg else
                            "xgmi-in-reduce-kernel" if xgmi is not None else
                            "xgmi-oneshot<=%dB+rccl" % comm.threshold) if routed is not None else
                 ("rccl" if comm is not None else ("gloo" if ctx.world_size > 1 else "none")))
    w.group = group
    if routed is not None:
        w.check = comm.xgmi.check  # raises if any one-shot call timed out waiting for a peer
    if mega is not None:
        def mega_check():
            if mega.errors():
                raise RuntimeError("MegaMLP: a grid barrier timed out (workgroups not co-resident)")

        w.check = mega_check

    def phase_step(i, timer):
        x, y = batch_fn(i)
        return train_step(x, y, timer)

    w.phase_step = phase_step
    w.phase_inputs = lambda: list(batch_fn(0))
    w.phase_call = lambda timer, x, y: train_step(x, y, timer)
    if fused is not None and ctx.world_size == 1:
        w.kernel_stamps = _cnn_kernel_stamps(fused, batch, dev)
    return w


def _cnn_kernel_stamps(fused, batch, dev):
    """(enable, summarize) of the fused CNN kernel's in-kernel phase stamps (100 MHz wall clock per workgroup;
    scripts/cnn_phase_stamps.py names them): the config-1 JSON explains its one graph phase by them."""
    names = ["P0_load", "P1_conv1", "P2_conv2", "P3_fc1", "P4a_fc2", "P4b_loss", "P5_fc2_bwd", "P6_fc1_bwd",
             "P7a_conv2_wgrad", "P7b_conv2_dgrad", "P9_conv1_wgrad"]

    def enable():
        fused.stamps = torch.zeros(fused._nwg(batch), 16, dtype=torch.long, device=dev)

    def summarize(t_start, t_end, hz):
        """Per-phase us of the last stamped replay: the phase's stamp kernels bracket [t_start, t_end]."""
        st = fused.stamps.cpu().double() * (1e6 / hz)  # us
        d = st[:, 1:12] - st[:, 0:11]
        med = {n: round(float(d[:, i].median()), 3) for i, n in enumerate(names)}
        wg_med = float((st[:, 11] - st[:, 0]).median())
        t0, t1 = t_start * 1e6 / hz, t_end * 1e6 / hz
        first, drained = float(st[:, 0].min()), float(st[:, 12].max())
        out = {"launch_to_first_workgroup": round(first - t0, 3)}
        out.update(med)
        out["workgroup_skew_and_drain"] = round(drained - first - wg_med, 3)
        out["reduce_sgd_kernel_and_boundaries"] = round(t1 - drained, 3)
        out["sum"] = round(sum(v for v in out.values()), 3)
        out["span"] = round(t1 - t0, 3)
        return out

    def disable():
        fused.stamps = None

    return enable, summarize, disable


def build_hvd_cnn(args, ctx, batch) -> Workload:
    """The reference's Horovod script (horovod/mnist_horovod.py:28-67) on the MI355X runtime; see the module
    docstring.  CPU: the autograd Net through the same optimizer wrapper, eager."""
    from .. import hvd
    from ..data.synthetic import SyntheticMNIST
    from ..models.cnn import Net
    from ..ops import functional as OF
    import math

    from ..ops.optim import FusedAdamW, FusedSGD

    elastic = args.model == "hvd_cnn_elastic"
    dev = ctx.device
    on_gpu = dev.type == "cuda"
    hvd.init(device="cpu" if not on_gpu else None)
    torch.manual_seed(0)
    model = Net().to(dev)
    data = SyntheticMNIST(max(8 * batch, 16384), device=dev, seed=hvd.rank())
    fused = grads = None
    if on_gpu:
        from ..models.cnn_fused import FusedCNN

        fused = FusedCNN(model)
        grads = fused.grad_buffer()  # p.grad = views of one flat buffer: the engine reduces it in place
        fused.always_prep = False  # AdamW: fused.adamw_step refreshes the fragments with the update
        if elastic:  # ... so the optimiser need not keep the layer path's bf16 layouts (hvd/cnn_step.py)
            for p in model.parameters():
                p.__dict__["_pde_own_copies"] = True
    inner = (FusedAdamW(model.parameters(), lr=0.01 / math.sqrt(hvd.size())) if elastic
             else FusedSGD(model.parameters(), lr=0.01))
    opt = hvd.DistributedOptimizer(inner, named_parameters=model.named_parameters())
    hvd.broadcast_parameters(model.state_dict(), root_rank=0)
    if fused is not None:
        fused.invalidate()
    world = hvd.size()

    def train_step(x, y):
        if fused is None:
            opt.zero_grad()
            loss = OF.nll_loss(model(x), y)
            loss.backward()
            opt.step()
            return loss
        if elastic:  # AdamW: the engine's all-reduce (graph mode: stream-ordered) + ONE update + fragment launch
            loss = fused.forward_backward(x, y, grad_out=grads)
            opt.synchronize()
            with opt.skip_synchronize():
                fused.adamw_step(opt, grads)
            return loss
        if world == 1:  # all-reduce = identity: the SGD update rides in the reduction kernel
            opt.synchronize()
            return fused.forward_backward(x, y, grad_out=grads, sgd=opt)
        loss = fused.forward_backward(x, y, grad_out=grads)
        opt.synchronize()  # engine (first step) / stream-ordered cached batches (graph mode)
        with opt.skip_synchronize():
            fused.sgd_step(opt, grads)  # opt.step(), fused with the conv-weight fragment refresh
        return loss

    def batch_fn(i):
        return data.batch(i, batch)

    one = group = None
    if on_gpu:
        train_step(*batch_fn(0))  # negotiated through the engine: every gradient enters the response cache
        torch.cuda.synchronize()
        opt.enable_graph_mode()
        if not args.no_graph:
            one, group = _capture(train_step, [batch_fn(j) for j in range(max(1, args.graph_steps))],
                                  args.graph_steps, ctx.rank)

    def step(i):
        x, y = batch_fn(i)
        return one(x, y) if one is not None else train_step(x, y)

    st = hvd.engine_stats()
    w = Workload(step, batch * world, f"dp{world}", hipgraph=one is not None, fused_step=fused is not None,
                 steps_per_graph=group.steps if group is not None else (1 if one is not None else 0),
                 api="horovod DistributedOptimizer + broadcast_parameters",
                 optimizer="adamw (FusedAdamW, lr 0.01/sqrt(size))" if elastic else "sgd (fused into the reduction)",
                 allreduce=("none (world 1)" if world == 1 else
                            f"fusion engine: {'xgmi-oneshot' if st.get('xgmi_batches') else st.get('backend')}"
                            f"{' graph mode' if on_gpu else ''}"))
    w.group = group

    keys = ("requests", "batches", "string_gathers", "bit_allreduces", "cache_hits", "cache_entries", "xgmi_batches",
            "rccl_batches", "inplace_batches", "inline_calls")
    marks = {}

    def mark():  # engine counters at the start of the timed region
        marks.update(hvd.engine_stats())

    def check():
        s2 = hvd.engine_stats()
        w.info["engine"] = {k: s2[k] for k in keys if k in s2}
        if marks:  # the timed region alone: in graph mode no negotiation cycle runs (bit_allreduces ~0)
            w.info["engine_timed_region"] = {k: s2[k] - marks.get(k, 0) for k in keys if k in s2}
        if s2.get("error"):
            raise RuntimeError(f"hvd engine error: {s2['error']}")

    w.check = check
    w.mark = mark
    w.close = hvd.shutdown
    return w


# The measured pipeline-unit table (scripts/pipeline_units.py --json over the stage benches of this round; a copy
# of profiles/r5_pipeline_units.json shipped with the package, so every GPU box has it): the default GPU unit size
# of resnet50_pp and the predicted-vs-1-GPU numbers its record carries.
UNIT_TABLE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "pipeline_units.json")


def _unit_table():
    try:
        with open(os.environ.get("PDE_PIPE_UNIT_TABLE", UNIT_TABLE)) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def build_pipeline(args, ctx, batch) -> Workload:
    """ResNet-50 split in 2 stages (one GPU each) x world/2 data-parallel replicas of each stage
    (:class:`..apps.hybrid_ps.ResNetPipelineDP`); the whole pipelined step is one hipGraph per rank."""
    from ..apps.hybrid_ps import ResNetPipelineDP

    on_gpu = ctx.device.type == "cuda"
    nranks = _data_plane_check(ctx, None)
    tab = _unit_table() if on_gpu else None
    mb_group, choice = args.mb_group, {"source": "--mb-group" if args.mb_group else None}
    if mb_group is None and os.environ.get("PDE_PIPE_MB_GROUP"):
        choice["source"] = "PDE_PIPE_MB_GROUP"
    elif mb_group is None and tab and tab.get("best"):
        mb_group = tab["best"]["mb_per_unit"]  # the measured best unit size
        choice["source"] = "measured table (best predicted 2-GPU rate)"
    pipe = ResNetPipelineDP(ctx, batch, args.split_size, args.image or 128, args.schedule, tag="bench",
                            mb_group=mb_group)
    if tab:
        row = next((r for r in tab["rows"] if r["mb_per_unit"] == pipe.mb_group), None)
        choice.update(table=tab.get("source_table", "profiles/r5_pipeline_units.json"),
                      formula=tab.get("formula"),
                      rows={r["mb_per_unit"]: r["predicted_2gpu_img_s"] for r in tab["rows"]},
                      predicted_2gpu_img_s=row["predicted_2gpu_img_s"] if row else None,
                      one_gpu_img_s=tab.get("one_gpu_img_s"))
    elif choice["source"] is None:
        choice["source"] = "no measured table: one unit per step on the GPU"
    one = None
    if not args.no_graph and pipe.capturable:
        one, _ = _capture(pipe.step, [()], 1, ctx.rank)

    def step(i):
        return one() if one is not None else pipe.step()

    w = Workload(step, pipe.images_per_step, f"pp{pipe.stages}xdp{pipe.dp}", hipgraph=one is not None,
                 fused_step=False, rccl_nranks=nranks, steps_per_graph=1 if one is not None else 0,
                 split_size=args.split_size, microbatches=batch // args.split_size, mb_per_unit=pipe.mb_group,
                 pipeline_units=pipe.n_mb, schedule=args.schedule, cross_stage_overlap=pipe.n_mb > 1,
                 unit_choice=choice, predicted_2gpu_img_s=choice.get("predicted_2gpu_img_s"),
                 one_gpu_img_s=choice.get("one_gpu_img_s"))
    w.loss_rank = pipe.stages - 1
    w.close = pipe.close
    w.check = pipe.check
    w.phase_step = lambda i, timer: pipe.step(timer)
    w.phase_inputs = lambda: []
    w.phase_call = lambda timer: pipe.step(timer)
    w.per_stage = True
    return w


def _secondary_pipeline(ctx, timeout_s: float = 420.0):
    """BASELINE configs 3/4 measured alongside the headline: after the CNN measurement, every rank launches
    one child process running ``bench.py --model resnet50_pp`` on the same GPU (a fresh process group on a new
    port; world 2 = the 2-stage pipeline, world 8 = pp2 x dp4).  Children are separate processes so a failure
    or hang there can never cost the headline line: each parent kills its child at ``timeout_s``."""
    import subprocess

    store = dist.distributed_c10d._get_default_store()
    if ctx.rank == 0:
        store.set("pde/bench/secondary_port", str(pdist.free_port()))
    port = store.get("pde/bench/secondary_port").decode()
    bench_py = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "bench.py")
    # a plain env:// job: drop torchrun's agent-store variables (TORCHELASTIC_USE_AGENT_STORE would make the
    # child's rank 0 connect to a store server that does not exist on the new port)
    env = {k: v for k, v in os.environ.items() if not k.startswith(("TORCHELASTIC_", "GROUP_", "ROLE_"))}
    env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=port, RANK=str(ctx.rank), WORLD_SIZE=str(ctx.world_size),
               LOCAL_RANK=str(ctx.local_rank), PDE_BENCH_CHILD="1")
    cmd = [sys.executable, bench_py, "--model", "resnet50_pp", "--gpus", str(ctx.world_size), "--steps", "20",
           "--warmup", "5"] + os.environ.get("PDE_BENCH_SECONDARY_ARGS", "").split()
    result = {"model": MODEL_NAMES["resnet50_pp"], "baseline_config": BASELINE_CONFIG["resnet50_pp"]}
    try:
        res = subprocess.run(cmd, env=env, timeout=timeout_s, capture_output=True, text=True)
        line = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
        if res.returncode != 0:
            result["error"] = f"rc={res.returncode}: " + res.stderr.strip().splitlines()[-1][:300] if res.stderr.strip() \
                else f"rc={res.returncode}"
        elif line:
            rec = json.loads(line[-1])
            result.update(value=rec["value"], unit=rec["unit"], ms_per_step=rec["ms_per_step"], steps=rec["steps"],
                          warmup=rec["warmup"], vs_baseline=rec["vs_baseline"],
                          parallelism=rec["config"]["parallelism"], hipgraph=rec["config"]["hipgraph"],
                          global_batch=rec["config"]["global_batch"], final_loss=rec["config"]["final_loss"],
                          split_size=rec["config"].get("split_size"), mb_per_unit=rec["config"].get("mb_per_unit"),
                          cross_stage_overlap=rec["config"].get("cross_stage_overlap"),
                          unit_choice=rec["config"].get("unit_choice"),
                          predicted_2gpu_img_s=rec["config"].get("predicted_2gpu_img_s"),
                          one_gpu_img_s=rec["config"].get("one_gpu_img_s"))
    except subprocess.TimeoutExpired:
        result["error"] = f"timeout after {timeout_s:.0f} s"
    except Exception as exc:  # noqa: BLE001 - never let the secondary measurement cost the headline
        result["error"] = repr(exc)[:300]
    return result


def run_steps(work: Workload, first: int, n: int):
    loss = None
    i = 0
    while work.group is not None and n - i >= work.group.steps:
        loss = work.group.replay()
        i += work.group.steps
    while i < n:
        loss = work.step(first + i)
        i += 1
    return loss


def _report_loss(work, ctx, loss):
    """The loss of the reporting rank (the last pipeline stage for resnet50_pp), as a float on rank 0."""
    t = torch.zeros(1, dtype=torch.float32, device=ctx.device)
    if loss is not None and ctx.rank == work.loss_rank:
        t.copy_(loss.detach().float().reshape(-1)[:1])
    if ctx.world_size > 1 and work.loss_rank != 0:
        dist.broadcast(t, work.loss_rank)
    return float(t.item())


PHASE_STEPS = 3


def _graph_phases(work, ctx, args):
    """Phases of the CAPTURED step: the workload's step with a :class:`GraphPhaseTimer` recorded into a fresh
    single-step hipGraph (every rank captures in lockstep: pipeline stages exchange inside it), replayed
    PHASE_STEPS times after the timed region."""
    from ..utils.graph import CapturedStep
    from ..utils.log import GraphPhaseTimer

    timer = GraphPhaseTimer(ctx.device)
    inputs = work.phase_inputs()
    ks = getattr(work, "kernel_stamps", None)
    if ks is not None:
        ks[0]()  # the captured kernels write their in-kernel phase stamps on every replay

    def fn(*xs):  # events only in the captured step, not in the capture's eager warm-up
        return work.phase_call(timer if torch.cuda.is_current_stream_capturing() else NO_PHASES, *xs)

    try:
        one = CapturedStep(fn, inputs, warmup=1).capture()
        for _ in range(PHASE_STEPS):
            one(*inputs)
            torch.cuda.synchronize()
            timer.replayed()
        out = timer.summary()
        if ks is not None:  # the one phase broken down by the kernel's own stamps (last replay)
            t = timer.buf[:2].tolist()
            out["kernel_us"] = ks[1](t[0], t[1], timer._hz)
    finally:
        if ks is not None:
            ks[2]()
    return out


def _region_overheads(work, ctx, reps: int = 5):
    """Where the fixed cost of a timed region goes: wall time of a region with 0 / 1 / 2
    multi-step graph replays between barrier + synchronize brackets (medians of ``reps``), after the timed region.
    One replay's device time = t(2) - t(1); the fixed cost = t(1) - that (graph launch, first-node latency,
    the synchronize); the host-side launch = time until replay() returns."""
    import statistics

    def region(n):
        pdist.barrier(ctx)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            work.group.replay()
        th = time.perf_counter()
        pdist.barrier(ctx)
        torch.cuda.synchronize()
        return time.perf_counter() - t0, th - t0

    res = {n: [region(n) for _ in range(reps)] for n in (0, 1, 2)}
    med = {n: statistics.median(r[0] for r in res[n]) * 1e3 for n in res}
    per = med[2] - med[1]
    return {"method": f"median of {reps} regions with 0/1/2 replays of the {work.group.steps}-step graph",
            "empty_region_ms": round(med[0], 4), "one_replay_region_ms": round(med[1], 4),
            "replay_device_ms": round(per, 4), "fixed_region_ms": round(med[1] - per, 4),
            "replay_host_launch_ms": round(statistics.median(r[1] for r in res[1]) * 1e3, 4)}


def _measure_phases(work, ctx, args):
    """Per-phase device milliseconds per step.  GPU runs with a captured step: timing events
    inside a captured copy of the benchmarked step (:func:`_graph_phases`), so the phases sum to the step's
    device time.  Otherwise (CPU, eager runs, or a capture failure): PHASE_STEPS eager steps after the timed
    region.  Data parallel: rank 0's phases.  Pipeline: one entry per stage of the first pipeline (fwd / bwd
    compute, recv_wait = time the stage's stream spends in receive kernels waiting for its neighbour, comm =
    stage all-reduce, opt)."""
    if not hasattr(work, "phase_step"):
        return None
    method = f"hipEvents, {PHASE_STEPS} eager steps after the timed region"
    local = None
    if ctx.device.type == "cuda" and work.info.get("hipgraph") and hasattr(work, "phase_call"):
        try:
            local = _graph_phases(work, ctx, args)
            method = (f"wall-clock stamp nodes at the phase boundaries of a captured single-step hipGraph, "
                      f"{PHASE_STEPS} replays")
        except Exception as exc:  # noqa: BLE001 - diagnostics never cost the headline line
            torch.cuda.synchronize()
            from .. import _native

            _native.C().clear_last_error()
            local = None
            method += f" (graph attribution failed: {repr(exc)[:120]})"
    if local is None:
        timer = PhaseTimer(ctx.device)
        try:
            for k in range(PHASE_STEPS):
                work.phase_step(args.warmup + args.steps + k, timer)
                timer.steps += 1
            local = timer.summary()
        except Exception as exc:  # noqa: BLE001 - diagnostics never cost the headline line
            local = {"error": repr(exc)[:200]}
    if getattr(work, "per_stage", False) and ctx.world_size > 1:
        allp = [None] * ctx.world_size
        dist.all_gather_object(allp, local)
        stages = [dict(stage=s, **allp[s]) for s in range(min(2, ctx.world_size))]
        return {"method": method, "stages": stages}
    return {"method": method, "rank0_ms": local}


def main(argv=None):
    args = parse_args(argv)
    if args.model == "elastic_cnn":  # BASELINE config 2 (bench/elastic.py); bench.py runs it without torchrun
        from . import elastic

        if args.elastic_worker:
            return elastic.worker(args)
        bench_py = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                "bench.py")
        sys.exit(elastic.parent(args, bench_py))
    batch = args.batch or DEFAULT_BATCH[args.model]
    ctx = pdist.init_distributed(device="cpu" if args.device == "cpu" else None)
    if args.gpus is not None and args.gpus != ctx.world_size:
        raise SystemExit(f"--gpus {args.gpus} but the job has {ctx.world_size} ranks (WORLD_SIZE); "
                         "run bench.py without torchrun to have it launch the ranks")
    on_gpu = ctx.device.type == "cuda"

    def sync():
        if on_gpu:
            torch.cuda.synchronize()

    if args.model == "resnet50_pp":
        work = build_pipeline(args, ctx, batch)
    elif args.model in ("hvd_cnn", "hvd_cnn_elastic"):
        work = build_hvd_cnn(args, ctx, batch)
    else:
        work = build_data_parallel(args, ctx, batch)
    run_steps(work, 0, args.warmup)
    pdist.barrier(ctx)
    sync()
    if hasattr(work, "mark"):
        work.mark()
    t0 = time.perf_counter()
    loss = run_steps(work, args.warmup, args.steps)
    pdist.barrier(ctx)
    sync()
    dt = time.perf_counter() - t0
    if hasattr(work, "check"):
        work.check()
    if on_gpu:  # a one-launch BatchNorm hand-off that timed out invalidates the measurement: fail loudly
        from ..ops.functional import check_device_errors

        check_device_errors(f"rank {ctx.rank} after the timed region")
    dt = pdist.max_over_ranks(dt, ctx.device)
    final_loss = _report_loss(work, ctx, loss)
    phases = _measure_phases(work, ctx, args) if os.environ.get("PDE_BENCH_PHASES", "1") != "0" else None
    overheads = None
    if on_gpu and work.group is not None and os.environ.get("PDE_BENCH_OVERHEADS", "1") != "0":
        try:
            overheads = _region_overheads(work, ctx)
        except Exception as exc:  # noqa: BLE001 - diagnostics never cost the headline line
            overheads = {"error": repr(exc)[:200]}
    value = work.images_per_step * args.steps / dt
    secondary = None
    mode = os.environ.get("PDE_BENCH_SECONDARY", "1")  # 0: off; force: also on CPU/gloo (plumbing tests)
    if (args.model == "cnn" and ctx.world_size >= 2 and ctx.world_size % 2 == 0 and mode != "0" and
            "PDE_BENCH_CHILD" not in os.environ and (mode == "force" or (on_gpu and ctx.backend == "nccl"))):
        secondary = _secondary_pipeline(ctx)
    same_shape = args.image is None and batch == DEFAULT_BATCH[args.model]
    ref = REFERENCE_IMG_S.get((args.model, ctx.world_size)) if same_shape else None
    if ctx.rank == 0:
        name = MODEL_NAMES[args.model] + (str(args.stage) if args.model == "resnet50_stage" else "")
        cfg = {"model": name, "baseline_config": BASELINE_CONFIG[args.model],
               "global_batch": work.images_per_step, "seq_len": None,
               "image": "1x28x28" if args.model in ("cnn", "hvd_cnn", "hvd_cnn_elastic", "mlp") else f"3x{args.image or 128}x{args.image or 128}",
               "parallelism": work.parallelism, "final_loss": round(final_loss, 4)}
        cfg.update(work.info)
        if phases is not None:
            cfg["phases"] = phases
        if overheads is not None:
            cfg["region_overheads"] = overheads
        if secondary is not None:
            cfg["secondary"] = secondary
        print(json.dumps({
            "metric": METRIC, "value": round(value, 1), "unit": "images/s", "n_gpus": ctx.world_size,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1000.0, 4),
            "higher_is_better": True, "scaling": "weak",
            "vs_baseline": round(value / ref, 2) if ref else None,
            "dtype": "bf16" if on_gpu else "fp32", "data": "synthetic (random init)", "config": cfg,
        }), flush=True)
    if hasattr(work, "close"):
        work.close()
    pdist.shutdown()
