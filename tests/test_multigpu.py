"""Multi-GPU data-plane tests at world N in {2, 4, 8}: one process per GPU over RCCL (xGMI on an MI355X
node).  Each test skips when the box has fewer than N GPUs (the 1-GPU rehearsal boxes); the same code
paths are exercised on gloo by the CPU suite and at world 1 by tests/test_comm_gpu.py.

Checks, per world size:
* the stream-ordered RCCL communicator (parallel/rccl.py) all-reduce against an fp32 sum of every
  rank's data, plus the rank count RCCL reports;
* the pipeline's per-direction P2P channel (parallel/pipeline.py) in both directions;
* the Horovod engine (negotiated fusion over RCCL) against the same fp32 sum;
* 2-stage pipeline gradients (gpipe and 1f1b, hipGraph-free) against a single-process reference;
* the one-shot xGMI peer all-reduce (csrc/comm/xgmi_allreduce.hip) against RCCL;
* the fused CNN step with that exchange folded into its reduction kernel against local gradients +
  RCCL all-reduce + the separate SGD launch (replicas bit-identical).
"""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_SCRIPT = r"""
import os, sys, torch, torch.distributed as dist
sys.path.insert(0, os.environ["REPO"])
from pytorch_distributed_examples_amd.parallel import dist as pdist
ctx = pdist.init_distributed()
N, r, dev = ctx.world_size, ctx.rank, ctx.device

def rank_data(k, n, seed):
    g = torch.Generator().manual_seed(seed * 1000 + k)
    return torch.randn(n, generator=g)

# 1. stream-ordered RCCL all-reduce vs fp32 sum
from pytorch_distributed_examples_amd.parallel.rccl import StreamComm
comm = StreamComm(dev)
assert comm.rccl.nranks() == N
for n in (1, 1000, 21840, 1 << 20):
    x = rank_data(r, n, n).to(dev)
    comm.allreduce_(x)
    ref = sum(rank_data(k, n, n) for k in range(N))
    torch.cuda.synchronize()
    assert torch.allclose(x.cpu(), ref, rtol=1e-5, atol=1e-5), n

# 2. per-direction P2P channels between pipeline neighbours (2k, 2k+1)
from pytorch_distributed_examples_amd.parallel.pipeline import P2PChannel
peer = r + 1 if r % 2 == 0 else r - 1
ch = P2PChannel(peer, "mgtest", dev)
a = torch.full((4096,), float(r), device=dev, dtype=torch.bfloat16)
for it in range(3):
    if r % 2 == 0:
        ch.send(a + it)
        got = ch.recv((4096,), torch.bfloat16)   # the opposite direction at the same time
    else:
        got = ch.recv((4096,), torch.bfloat16)
        ch.send(a + it)
    ch.flush()
    torch.cuda.synchronize()
    assert torch.all(got.float() == float(peer + it)), (it, got[:4])
ch.close()

# 3. Horovod engine: negotiated, fused, RCCL
from pytorch_distributed_examples_amd import hvd
hvd.init()
ts = [rank_data(r, n, 7 + i).to(dev) for i, n in enumerate((3, 1000, 17, 4096))]
order = range(len(ts)) if r % 2 == 0 else reversed(range(len(ts)))
hs = {i: hvd.allreduce_async_(ts[i], name=f"t{i}", op=hvd.Sum) for i in order}
for i in range(len(ts)):
    hvd.synchronize(hs[i])
torch.cuda.synchronize()
for i, n in enumerate((3, 1000, 17, 4096)):
    ref = sum(rank_data(k, n, 7 + i) for k in range(N))
    assert torch.allclose(ts[i].cpu(), ref, rtol=1e-5, atol=1e-5), i
hvd.shutdown()

# 4. one-shot xGMI peer all-reduce vs RCCL (small, latency-bound buckets)
from pytorch_distributed_examples_amd.parallel.xgmi_allreduce import XgmiAllreduce
xa = XgmiAllreduce(dev, max_bytes=4 << 20)
for n in (1, 5, 21840, 262144):
    x = rank_data(r, n, 99 + n).to(dev)
    y = x.clone()
    xa.allreduce_(x, avg=False)
    comm.allreduce_(y)
    torch.cuda.synchronize()
    ref = sum(rank_data(k, n, 99 + n) for k in range(N))
    assert torch.allclose(x.cpu(), ref, rtol=1e-5, atol=1e-5), n
    # every rank sums in rank order: bit-identical results on every rank
    gathered = [torch.empty_like(x) for _ in range(N)]
    dist.all_gather(gathered, x)
    for gth in gathered:
        assert torch.equal(gth, x)
# 5. fused CNN with the exchange inside its reduction kernel vs local gradients + RCCL all-reduce + SGD launch
from pytorch_distributed_examples_amd.models.cnn import Net
from pytorch_distributed_examples_amd.models.cnn_fused import FusedCNN
from pytorch_distributed_examples_amd.ops.optim import FusedSGD
torch.manual_seed(0)
net_a, net_b = Net().to(dev), Net().to(dev)
net_b.load_state_dict(net_a.state_dict())
fa, fb = FusedCNN(net_a), FusedCNN(net_b)
oa, ob = FusedSGD(net_a.parameters(), lr=0.05), FusedSGD(net_b.parameters(), lr=0.05)
ga, gb = fa.grad_buffer(), fb.grad_buffer()
gen = torch.Generator().manual_seed(100 + r)
for it in range(3):
    x = torch.randn(512, 1, 28, 28, generator=gen).to(dev)
    y = torch.randint(0, 10, (512,), generator=gen).to(dev)
    fa.forward_backward(x, y, grad_out=ga, sgd=oa, xgmi=xa, p_drop2=0.0, p_drop1=0.0)
    fb.forward_backward(x, y, grad_out=gb, p_drop2=0.0, p_drop1=0.0)
    comm.allreduce_(gb)
    gb.mul_(1.0 / N)
    fb.sgd_step(ob, gb)
torch.cuda.synchronize()
xa.check()
assert torch.allclose(ga, gb, rtol=1e-4, atol=1e-6), (ga - gb).abs().max()
assert torch.allclose(fa.flat, fb.flat, rtol=1e-4, atol=1e-6), (fa.flat - fb.flat).abs().max()
gathered = [torch.empty_like(fa.flat) for _ in range(N)]
dist.all_gather(gathered, fa.flat)
for gth in gathered:
    assert torch.equal(gth, fa.flat)  # bit-identical replicas
xa.close()
comm.destroy()
dist.destroy_process_group()
print("MULTIGPU_OK", r)
"""

_PIPE = r"""
import os, sys, copy, torch, torch.distributed as dist
sys.path.insert(0, os.environ["REPO"])
from torch import nn
from pytorch_distributed_examples_amd.parallel import dist as pdist
from pytorch_distributed_examples_amd.parallel.pipeline import PipelineEngine
ctx = pdist.init_distributed()
r, dev = ctx.rank, ctx.device
torch.manual_seed(0)
s0 = nn.Sequential(nn.Linear(64, 128), nn.ReLU()).to(dev)
s1 = nn.Linear(128, 16).to(dev)
full = nn.Sequential(copy.deepcopy(s0), copy.deepcopy(s1))
stage = r % 2
mod = s0 if stage == 0 else s1
for sched in ("gpipe", "1f1b"):
    for p in mod.parameters():
        p.grad = None
    eng = PipelineEngine(mod, stage, 2, r - 1 if stage else None, r + 1 if stage == 0 else None, dev,
                         loss_fn=lambda a, b: ((a - b) ** 2).mean(), schedule=sched, tag="mg" + sched)
    g = torch.Generator().manual_seed(5)
    x, y = torch.randn(32, 64, generator=g).to(dev), torch.randn(32, 16, generator=g).to(dev)
    loss = eng.train_step(list(x.split(8)) if stage == 0 else None, list(y.split(8)) if stage == 1 else None, 4)
    for p in full.parameters():
        p.grad = None
    ref = ((full(x) - y) ** 2).mean()
    ref.backward()
    refmod = full[0] if stage == 0 else full[1]
    for p, q in zip(mod.parameters(), refmod.parameters()):
        assert torch.allclose(p.grad, q.grad, atol=1e-5, rtol=1e-4), sched
    if stage == 1:
        assert abs(loss.item() - ref.item()) < 1e-5
    eng.close()
dist.destroy_process_group()
print("PIPE_OK", r)
"""


def _torchrun(script, n):
    import tempfile

    from pytorch_distributed_examples_amd.parallel.dist import free_port

    env = dict(os.environ, REPO=REPO)
    env.pop("PDE_BACKEND", None)
    with tempfile.NamedTemporaryFile("w", suffix=".py", delete=False) as f:
        f.write(script)
        path = f.name
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), path]
    try:
        return subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    finally:
        os.unlink(path)


@pytest.mark.parametrize("n", [2, 4, 8])
def test_data_plane_world_n(gpu, n):
    if torch.cuda.device_count() < n:
        pytest.skip(f"needs {n} GPUs, box has {torch.cuda.device_count()}")
    res = _torchrun(_SCRIPT, n)
    assert res.returncode == 0 and res.stdout.count("MULTIGPU_OK") == n, (res.stdout[-3000:], res.stderr[-5000:])


@pytest.mark.parametrize("n", [2, 4, 8])
def test_pipeline_grads_world_n(gpu, n):
    if torch.cuda.device_count() < n:
        pytest.skip(f"needs {n} GPUs, box has {torch.cuda.device_count()}")
    res = _torchrun(_PIPE, n)
    assert res.returncode == 0 and res.stdout.count("PIPE_OK") == n, (res.stdout[-3000:], res.stderr[-5000:])


_RESNET_PP = r"""
import os, sys, torch, torch.distributed as dist
sys.path.insert(0, os.environ["REPO"])
from pytorch_distributed_examples_amd.parallel import dist as pdist
from pytorch_distributed_examples_amd.apps.hybrid_ps import ResNetPipelineDP
from pytorch_distributed_examples_amd.utils.graph import CapturedStep
ctx = pdist.init_distributed()
N, r, dev = ctx.world_size, ctx.rank, ctx.device
for schedule in ("gpipe", "1f1b"):
    torch.manual_seed(0)
    pipe = ResNetPipelineDP(ctx, batch=16, split_size=4, image=64, schedule=schedule, lr=0.02, tag="mg" + schedule)
    assert pipe.capturable, "BASELINE configs 3/4: the whole pipelined step is one hipGraph per rank"
    graph = CapturedStep(pipe.step, [], warmup=1).capture()
    losses = [float(graph().item()) for _ in range(4)]
    pipe.check()
    flat = torch.cat([p.detach().float().reshape(-1) for p in pipe.module.parameters()])
    assert torch.isfinite(flat).all()
    # every data-parallel replica of a stage holds bit-identical weights (stage all-reduce, bf16 wire, overlapped)
    gathered = [torch.empty_like(flat) for _ in range(N)]
    dist.all_gather(gathered, flat)
    for k in range(r % 2, N, 2):
        assert torch.equal(gathered[k], flat), (schedule, r, k)
    if r % 2 == 1:
        assert all(l == l and l < 1e3 for l in losses), losses
    pipe.close()
dist.destroy_process_group()
print("RESNET_PP_OK", r)
"""


@pytest.mark.parametrize("n", [2, 4, 8])
def test_resnet_pipeline_dp_world_n(gpu, n):
    """BASELINE configs 3 (n=2) and 4 (n=8: pp2 x dp4): ResNetPipelineDP captured in a hipGraph, stage
    activations over the P2P ring, stage gradients all-reduced (bf16 wire, overlapped with the last
    micro-batch's backward) -- replicas must stay bit-identical, for gpipe and 1f1b."""
    if torch.cuda.device_count() < n:
        pytest.skip(f"needs {n} GPUs, box has {torch.cuda.device_count()}")
    res = _torchrun(_RESNET_PP, n)
    assert res.returncode == 0 and res.stdout.count("RESNET_PP_OK") == n, (res.stdout[-3000:], res.stderr[-5000:])


def test_resnet_rpc_two_gpus(gpu):
    """rpc/model_parallel_ResNet50.py with each stage on its own GPU (master + 2 stage workers)."""
    if torch.cuda.device_count() < 2:
        pytest.skip("needs 2 GPUs")
    env = dict(os.environ)
    env.pop("PDE_BACKEND", None)
    cmd = [sys.executable, os.path.join(REPO, "rpc", "model_parallel_ResNet50.py"), "--splits", "4", "8",
           "--num-batches", "3", "--verbose"]
    res = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert res.returncode == 0, (res.stdout[-3000:], res.stderr[-3000:])
    assert "number of splits = 8, execution time" in res.stdout, res.stdout
