#!/usr/bin/env python3
"""Headline benchmark: images/sec for the whole node (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--model cnn|mlp|resnet50] [--batch B]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Default workload = BASELINE.json configs[1]: "MNIST CNN DDP bf16 on N x MI355X, RCCL allreduce over
xGMI": the reference's MNIST CNN (horovod/mnist_horovod.py:9-25) at the reference's per-worker batch
(1024, :44), SGD lr 0.01 (:50), NLL loss on log_softmax, synthetic MNIST resident in HBM, random init.
One rank per GPU; per-GPU batch fixed (weak scaling).  Every timed step is a full training step:
forward, backward, gradient all-reduce (RCCL, xGMI-sized buckets), fused optimizer update.

W warmup steps are untimed; then K steps are timed between barrier+synchronize pairs and the MAX time
over ranks is reported.  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

os.environ.setdefault("OMP_NUM_THREADS", "1")

import torch  # noqa: E402

REPO = os.path.dirname(os.path.abspath(__file__))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

from pytorch_distributed_examples_amd.parallel import dist as pdist  # noqa: E402

# Reference numbers (CPU measurements of the reference -- no published figures).
BASELINE_IMG_S = {"mlp": 7452.0}  # world-1 MLP DDP; the CNN/ResNet configs have no reference number


def build(model_name: str, device, batch: int):
    from pytorch_distributed_examples_amd.ops import functional as OF
    from pytorch_distributed_examples_amd.ops.optim import FusedAdam, FusedSGD

    if model_name == "cnn":
        from pytorch_distributed_examples_amd.data.synthetic import SyntheticMNIST
        from pytorch_distributed_examples_amd.models.cnn import Net

        model = Net().to(device)
        data = SyntheticMNIST(max(8 * batch, 16384), device=device, seed=0)
        opt = FusedSGD(model.parameters(), lr=0.01)

        def batch_fn(i):
            return data.batch(i, batch)

        loss_fn = OF.nll_loss
    elif model_name == "mlp":
        from pytorch_distributed_examples_amd.data.synthetic import SyntheticMNIST
        from pytorch_distributed_examples_amd.models.mlp import reference_mlp

        model = reference_mlp().to(device)
        data = SyntheticMNIST(max(8 * batch, 16384), device=device, seed=0)
        opt = FusedAdam(model.parameters(), lr=1e-3)

        def batch_fn(i):
            return data.batch(i, batch)

        loss_fn = OF.cross_entropy
    elif model_name == "resnet50":
        from pytorch_distributed_examples_amd.data.synthetic import resnet_batch
        from pytorch_distributed_examples_amd.models.resnet import ResNet50

        model = ResNet50().to(device)
        g = torch.Generator().manual_seed(0)
        batches = [resnet_batch(batch, 128, 1000, device, g) for _ in range(2)]
        opt = FusedSGD(model.parameters(), lr=0.05)

        def batch_fn(i):
            return batches[i % 2]

        loss_fn = OF.mse_loss
    else:
        raise ValueError(model_name)
    return model, opt, batch_fn, loss_fn


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--model", default="cnn", choices=["cnn", "mlp", "resnet50"])
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch")
    ap.add_argument("--no-graph", action="store_true", help="run the step eagerly (no hipGraph capture)")
    ap.add_argument("--graph-steps", type=int, default=10,
                    help="consecutive training steps recorded into one hipGraph (each reads its own batch)")
    ap.add_argument("--generic", action="store_true", help="CNN: layer-by-layer kernels instead of the fused step")
    ap.add_argument("--device", default="auto", choices=["auto", "cpu"], help="cpu: contract/plumbing check only")
    args = ap.parse_args()
    batch = args.batch or {"cnn": 1024, "mlp": 128, "resnet50": 32}[args.model]

    ctx = pdist.init_distributed(device="cpu" if args.device == "cpu" else None)
    on_gpu = ctx.device.type == "cuda"

    def sync():
        if on_gpu:
            torch.cuda.synchronize()

    from pytorch_distributed_examples_amd.parallel.ddp import DistributedDataParallel

    model, opt, batch_fn, loss_fn = build(args.model, ctx.device, batch)
    # hipGraph capture needs capturable collectives: RCCL (or none at world 1), not gloo
    use_graph = not args.no_graph and on_gpu and (ctx.world_size == 1 or ctx.backend == "nccl")
    # GPU data plane for world > 1: our stream-ordered RCCL communicator (c10d's ProcessGroupNCCL aborts
    # the process when its work is captured into a hipGraph on ROCm -- parallel/rccl.py)
    comm = None
    if on_gpu and ctx.world_size > 1 and ctx.backend == "nccl":
        from pytorch_distributed_examples_amd.parallel.rccl import StreamComm

        comm = StreamComm(ctx.device)
    fused = None
    if args.model == "cnn" and not args.generic and ctx.device.type == "cuda":
        # whole-network fused kernel (csrc/kernels/cnn_fused.hip): gradients land directly in the
        # DDP flat buffer (forward layout), then one RCCL all-reduce and one fused SGD launch that also
        # refreshes the kernel's bf16 weight fragments (world 1: the SGD runs inside the slab reduction).
        from pytorch_distributed_examples_amd.models.cnn_fused import FusedCNN

        fused = FusedCNN(model)
        ddp = DistributedDataParallel(model, overlap=False, param_order="forward", comm=comm)
    else:
        ddp = DistributedDataParallel(model, overlap=not use_graph, comm=comm)

    def train_step(x, y):
        if fused is not None:
            if ctx.world_size == 1:  # SGD + weight-fragment refresh inside the slab reduction
                return fused.forward_backward(x, y, grad_out=ddp.flat_grad, sgd=opt)
            loss = fused.forward_backward(x, y, grad_out=ddp.flat_grad)
            ddp.sync_gradients()
            fused.sgd_step(opt, ddp.flat_grad)  # SGD + weight-fragment refresh, one launch
            return loss
        ddp.zero_grad()
        loss = loss_fn(ddp(x), y)
        loss.backward()
        if use_graph:
            ddp.sync_gradients()
        opt.step()
        return loss

    graphed = None
    group = None
    if use_graph:
        from pytorch_distributed_examples_amd.utils.graph import CapturedStep, CapturedSteps

        try:
            graphed = CapturedStep(train_step, batch_fn(0), warmup=3).capture()
            if args.graph_steps > 1:
                # G complete steps per replay, step j of the group reading dataset batch j in place:
                # one host launch per G steps instead of one per step (the MNIST step is ~50 us of GPU work)
                group = CapturedSteps(train_step, [batch_fn(j) for j in range(args.graph_steps)],
                                      warmup=1).capture()
        except Exception as exc:  # capture unsupported (e.g. collective in capture): run eagerly
            if ctx.rank == 0:
                print(f"[bench] hipGraph capture failed, running eagerly: {exc}", file=sys.stderr)
            from pytorch_distributed_examples_amd import _native

            torch.cuda.synchronize()
            _native.C().clear_last_error()  # the aborted capture leaves a sticky "last error" behind
            use_graph = False
            graphed = group = None
            if fused is None:  # the fused path keeps its forward-order, non-overlapped flat buffer
                ddp.remove_hooks()
                ddp = DistributedDataParallel(model, overlap=True, comm=comm)

    def step(i):
        x, y = batch_fn(i)
        return graphed(x, y) if graphed is not None else train_step(x, y)

    def run(first, n):
        """n full training steps starting at step index ``first``; returns the last loss."""
        loss = None
        i = 0
        while group is not None and n - i >= group.steps:
            loss = group.replay()
            i += group.steps
        while i < n:
            loss = step(first + i)
            i += 1
        return loss

    run(0, args.warmup)
    pdist.barrier(ctx)
    sync()
    t0 = time.perf_counter()
    loss = run(args.warmup, args.steps)
    pdist.barrier(ctx)
    sync()
    dt = time.perf_counter() - t0
    dt = pdist.max_over_ranks(dt, ctx.device)
    final_loss = float(loss.item())
    ms = dt / args.steps * 1000.0
    value = batch * ctx.world_size * args.steps / dt
    base = BASELINE_IMG_S.get(args.model)
    if ctx.rank == 0:
        print(json.dumps({
            "metric": "images/sec (whole node) MNIST DDP + ResNet50 RPC-MP at 1/2/4/8 MI355X",
            "value": round(value, 1),
            "unit": "images/s",
            "n_gpus": ctx.world_size,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / base, 2) if base else None,
            "dtype": "bf16",
            "data": "synthetic",
            "config": {"model": {"cnn": "mnist_cnn_Net", "mlp": "mnist_mlp_5x1024",
                                 "resnet50": "resnet50_128px"}[args.model],
                       "global_batch": batch * ctx.world_size, "seq_len": None,
                       "image": "1x28x28" if args.model != "resnet50" else "3x128x128",
                       "parallelism": f"dp{ctx.world_size}", "final_loss": round(final_loss, 4),
                       "hipgraph": graphed is not None, "fused_step": fused is not None,
                       "steps_per_graph": group.steps if group is not None else (1 if graphed is not None else 0)},
        }), flush=True)
    pdist.shutdown()


if __name__ == "__main__":
    main()
