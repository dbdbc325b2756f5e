"""One-shot peer all-reduce (csrc/comm/xgmi_allreduce.hip) rehearsed on ONE GPU: 2 and 4 processes share
the card, each maps the others' IPC-exported staging buffers exactly as the ranks of an 8-GPU node map
their peers' over xGMI.  Checks the result against an fp32 reference, bit-identity across ranks, the
hipGraph-captured form (epochs advance on every replay), a late peer (bounded spin, no timeout), and the
DDP routing communicator.  The N-GPU form against RCCL is in tests/test_multigpu.py."""
import os
import subprocess
import sys
import tempfile

import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_SCRIPT = r"""
import os, sys, time, torch, torch.distributed as dist
sys.path.insert(0, os.environ["REPO"])
from pytorch_distributed_examples_amd.parallel import dist as pdist
from pytorch_distributed_examples_amd.parallel.xgmi_allreduce import XgmiAllreduce
ctx = pdist.init_distributed()          # PDE_BACKEND=gloo: several ranks on one GPU
N, r, dev = ctx.world_size, ctx.rank, ctx.device

def rank_data(k, n, seed):
    g = torch.Generator().manual_seed(seed * 1000 + k)
    return torch.randn(n, generator=g)

xa = XgmiAllreduce(dev, max_bytes=4 << 20, timeout_s=20.0)
for n in (1, 7, 1000, 21840, 262144, 1 << 20):
    x = rank_data(r, n, n).to(dev)
    xa.allreduce_(x)
    torch.cuda.synchronize()
    ref = sum(rank_data(k, n, n) for k in range(N))
    assert torch.allclose(x.cpu(), ref, rtol=1e-5, atol=1e-5), n
    xs = [torch.empty(n) for _ in range(N)]
    dist.all_gather(xs, x.cpu())
    assert all(torch.equal(v, xs[0]) for v in xs), n
# unaligned views (scalar path) and averaging
big = rank_data(r, 1001, 5).to(dev)
v = big[1:]
xa.allreduce_(v, avg=True)
torch.cuda.synchronize()
ref = sum(rank_data(k, 1001, 5) for k in range(N))[1:] / N
assert torch.allclose(v.cpu(), ref, rtol=1e-5, atol=1e-6)
# a late peer: the others spin (bounded) until it arrives
if r == N - 1:
    time.sleep(0.3)
x = torch.full((4096,), float(r + 1), device=dev)
xa.allreduce_(x)
torch.cuda.synchronize()
assert torch.all(x == N * (N + 1) / 2)
# hipGraph: 3 all-reduces per replay, 4 replays; every replay advances the epochs
t = torch.full((21840,), float(r + 1), device=dev)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    for _ in range(3):
        t.mul_(0.5)
        xa.allreduce_(t)
vals = [float(k + 1) for k in range(N)]
t.fill_(float(r + 1))
for _ in range(4):
    g.replay()
    for _ in range(3):
        s = sum(0.5 * v for v in vals)
        vals = [s] * N
torch.cuda.synchronize()
assert torch.allclose(t, torch.full_like(t, vals[0]), rtol=1e-6), (t[:4], vals[0])
xa.check()
# DDP over the routing communicator: the small bucket takes the xGMI path
from pytorch_distributed_examples_amd.parallel.ddp import DistributedDataParallel
from pytorch_distributed_examples_amd.parallel.xgmi_allreduce import RoutedComm
class _Gloo:  # stand-in for the RCCL StreamComm (RCCL refuses 2 ranks on one GPU)
    size, rank, supports_avg = N, r, False
    def allreduce_async(self, t, avg=False):
        h = t.cpu(); dist.all_reduce(h); t.copy_(h / N if avg else h)
        class W:
            def wait(self): return True
        return W()
    def broadcast_(self, t, src):
        h = t.cpu(); dist.broadcast(h, src); t.copy_(h); return t
    def destroy(self): pass
comm = RoutedComm(_Gloo(), xa, threshold_bytes=1 << 20)
torch.manual_seed(r)
m = torch.nn.Linear(16, 8).to(dev)
ddp = DistributedDataParallel(m, overlap=False, comm=comm)
ddp.zero_grad()
ddp.flat_grad.fill_(float(r))
ddp.sync_gradients()
torch.cuda.synchronize()
assert torch.allclose(ddp.flat_grad, torch.full_like(ddp.flat_grad, (N - 1) / 2)), ddp.flat_grad[:4]
assert comm.routed["xgmi"] >= 1
xa.check()
dist.barrier()
xa.close()
dist.destroy_process_group()
print("XGMI_OK", r)
"""


def _run(n):
    from pytorch_distributed_examples_amd.parallel.dist import free_port

    env = dict(os.environ, REPO=REPO, PDE_BACKEND="gloo")
    with tempfile.NamedTemporaryFile("w", suffix=".py", delete=False) as f:
        f.write(_SCRIPT)
        path = f.name
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), path]
    try:
        return subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    finally:
        os.unlink(path)


@pytest.mark.parametrize("n", [2, 4])
def test_xgmi_oneshot_rehearsal_one_gpu(gpu, n):
    res = _run(n)
    assert res.returncode == 0 and res.stdout.count("XGMI_OK") == n, (res.stdout[-3000:], res.stderr[-6000:])


def test_xgmi_world1(gpu):
    """World 1: no peers, the call is a scale (avg) or identity."""
    from pytorch_distributed_examples_amd import _native

    C = _native.comm()
    xa = C.XgmiAllreduce(0, 1, gpu.index, 1 << 20)
    t = torch.arange(1000, dtype=torch.float32, device=gpu)
    xa.allreduce_(t, 0.5)
    torch.cuda.synchronize()
    assert torch.equal(t.cpu(), torch.arange(1000, dtype=torch.float32) * 0.5)
    assert xa.error() == 0
    xa.close()
