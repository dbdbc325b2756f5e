"""RPC model-parallel ResNet-50 (reference: rpc/model_parallel_ResNet50.py).

Kept from the reference: one master + 2 stage workers spawned with ``mp.spawn`` (:256-260), the stage
split (stem+layer1+layer2 | layer3+layer4+fc, :85-139), ``DistResNet50(split_size, ["worker1",
"worker2"])`` (:142-184) whose ``split_size`` is the micro-batch SIZE (quirk Q2), ``MSELoss`` against
one-hot labels of 1000 classes on ``randn(32,3,128,128)`` batches (:191-217), distributed autograd +
``DistributedOptimizer(SGD, lr=0.05)`` (:202-225), and the ``number of splits = ..., execution time = ...``
line for split sizes 4 and 8 (:258-262).

MI355X-first: stage k lives on GPU k-1 (NHWC bf16 MFMA kernels), the stage-1 -> stage-2 activation
(m x 16 x 16 x 512 bf16) moves GPU->GPU over xGMI (the IPC receive ring of csrc/comm/p2p_ring.hip; RCCL
send/recv with ``PDE_P2P=rccl``) instead of ``to_here()`` through the CPU; the
``Forward 2`` print (quirk Q12) is behind ``--verbose``.  A separate port is used per spawn (the reference
reuses 29500 for both spawns).
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

from ..models.resnet import ResNetShard1, ResNetShard2
from ..parallel.dist import free_ports
from ..rpc import DistributedOptimizer, RemotePipeline, dist_autograd
from ..utils import config as rtconfig
from ..utils.config import add_runtime_args

NUM_CLASSES = 1000


class DistResNet50(RemotePipeline):
    """Same constructor/forward/parameter_rrefs surface as the reference's DistResNet50 (:142-184)."""

    def __init__(self, split_size, workers, devices, mb_group=None):
        # mb_group: micro-batches per pipeline unit with per-micro-batch (grouped) BatchNorm (RemotePipeline)
        super().__init__(split_size, workers, [ResNetShard1, ResNetShard2], devices, mb_group=mb_group)


def run_master(split_size, args, devices):
    model = DistResNet50(split_size, ["worker1", "worker2"], devices, mb_group=args.mb_group)
    loss_fn = nn.MSELoss()
    opt = DistributedOptimizer(optim.SGD, model.parameter_rrefs(), lr=0.05)
    one_hot_indices = torch.LongTensor(args.batch_size).random_(0, NUM_CLASSES).view(args.batch_size, 1)
    times = []
    for i in range(args.num_batches):
        print(f"Processing batch {i}", flush=True)
        t0 = time.perf_counter()
        inputs = torch.randn(args.batch_size, 3, args.image_w, args.image_h)
        labels = torch.zeros(args.batch_size, NUM_CLASSES).scatter_(1, one_hot_indices, 1)
        with dist_autograd.context() as context_id:
            outputs = model(inputs)
            loss = loss_fn(outputs, labels)
            dist_autograd.backward(context_id, [loss])
            opt.step(context_id)
        times.append(time.perf_counter() - t0)
        if args.verbose:
            print(f"batch {i}: loss {loss.item():.5f} step {times[-1] * 1e3:.1f} ms", flush=True)
    steady = times[1:] if len(times) > 1 else times
    print(f"steady-state {args.batch_size * len(steady) / sum(steady):.1f} images/s "
          f"({sum(steady) / len(steady) * 1e3:.1f} ms/batch)", flush=True)


def run_worker(rank, world_size, num_split, args, rpc_port, pg_port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(rpc_port)
    options = rpc.TensorPipeRpcBackendOptions(num_worker_threads=16, rpc_timeout=300)
    use_gpu = torch.cuda.is_available() and not args.cpu
    ngpu = torch.cuda.device_count() if use_gpu else 0
    devices = [f"cuda:{i % ngpu}" if use_gpu else "cpu" for i in range(world_size - 1)]
    if rank == 0:
        rpc.init_rpc("master", rank=rank, world_size=world_size, rpc_backend_options=options)
        run_master(num_split, args, devices)
    else:
        # stage workers: their own process group for the RCCL / gloo data plane (ranks 0..S-1)
        if use_gpu:
            torch.cuda.set_device(devices[rank - 1])
        else:
            # CPU configuration: split the cores between the stage processes (each stage computes in
            # its executor thread; oversubscribed OpenMP teams spin against each other otherwise)
            torch.set_num_threads(max(1, (os.cpu_count() or 2) // (world_size - 1)))
        # PDE_BACKEND=gloo: both stages on one GPU (rehearsal); the stage data plane is the P2P ring either way
        dist.init_process_group(os.environ.get("PDE_BACKEND") or ("nccl" if use_gpu else "gloo"),
                                init_method=f"tcp://127.0.0.1:{pg_port}", rank=rank - 1, world_size=world_size - 1)
        rpc.init_rpc(f"worker{rank}", rank=rank, world_size=world_size, rpc_backend_options=options)
    rpc.shutdown()
    if rank != 0:
        dist.destroy_process_group()


def main(argv=None):
    ap = argparse.ArgumentParser(description="RPC model-parallel ResNet-50 over MI355X")
    ap.add_argument("--splits", type=int, nargs="+", default=[4, 8], help="micro-batch sizes (reference: 4 8)")
    ap.add_argument("--num-batches", type=int, default=3)
    ap.add_argument("--batch-size", type=int, default=32)
    ap.add_argument("--image-w", type=int, default=128)
    ap.add_argument("--image-h", type=int, default=128)
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--mb-group", type=int, default=None,
                    help="micro-batches per pipeline unit (grouped BatchNorm); default: all on GPUs, 1 on CPU")
    add_runtime_args(ap)
    args = ap.parse_args(argv)
    _cfg = rtconfig.apply(rtconfig.from_args(args))
    if hasattr(args, "device"):
        args.device = rtconfig.device_for(_cfg, args.device)
    world_size = 3
    for num_split in args.splits:
        tik = time.time()
        mp.spawn(run_worker, args=(world_size, num_split, args, *free_ports(2)), nprocs=world_size,
                 join=True)
        tok = time.time()
        print(f"number of splits = {num_split}, execution time = {tok - tik}", flush=True)
