"""GPU communication runtime on one MI355X: the RCCL communicator wrapper (csrc/comm/comm_manager.cpp),
the fusion engine's GPU path (pack kernel -> RCCL all-reduce -> unpack, csrc/comm/pack.hip) and the
Horovod-compatible API on top of it, world size 1 (multi-rank behaviour is covered on gloo by
tests/test_hvd_cpu.py; the driver's 8-GPU bench exercises RCCL across ranks)."""
import os
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_rccl_comm_world1(gpu):
    from pytorch_distributed_examples_amd import _native

    C = _native.comm()
    assert C.rccl_version() >= 22000
    comm = C.RcclComm()
    comm.init(C.rccl_unique_id(), 0, 1, gpu.index, True)
    t = torch.arange(1000, device=gpu, dtype=torch.float32)
    comm.allreduce_(t, 0)
    torch.cuda.synchronize()
    assert torch.equal(t.cpu(), torch.arange(1000, dtype=torch.float32))
    b = torch.randn(77, device=gpu, dtype=torch.bfloat16)
    ref = b.clone()
    comm.broadcast_(b, 0)
    g = comm.allgather(b)
    torch.cuda.synchronize()
    assert torch.equal(g.view(-1), ref.view(-1))
    comm.destroy()


def test_hvd_gpu_fusion_world1(gpu):
    from pytorch_distributed_examples_amd import hvd
    from pytorch_distributed_examples_amd.models.cnn import Net
    from pytorch_distributed_examples_amd.ops import functional as OF

    hvd.init()
    try:
        assert hvd.size() == 1 and hvd.rocm_built()
        # many small tensors of mixed sizes -> fused into one pack / all-reduce / unpack
        ts = [torch.randn(n, device=gpu) for n in (3, 1000, 17, 4096, 1, 513)]
        refs = [t.clone() for t in ts]
        hs = [hvd.allreduce_async_(t, name=f"t{i}", op=hvd.Sum, prescale_factor=2.0, postscale_factor=0.25)
              for i, t in enumerate(ts)]
        for h in hs:
            hvd.synchronize(h)
        for t, r in zip(ts, refs):
            assert torch.allclose(t, r * 0.5, atol=1e-6)
        st = hvd.engine_stats()
        assert st["fused_requests"] >= 5, st
        # bf16 wire compression round-trips through the pack kernel's f32->bf16 path
        x = torch.randn(2048, device=gpu)
        y = hvd.allreduce(x, op=hvd.Average, compression=hvd.Compression.bf16)
        # one bf16 rounding: |err| <= half an ulp = |x| * 2^-8 (randn draws beyond |x| = 4 exceed any fixed 1e-2)
        assert bool(((y - x).abs() <= x.abs() * 2.0 ** -8 + 1e-12).all())
        a, b = torch.randn(300, device=gpu), torch.randn(5000, device=gpu)
        ra, rb = a.clone(), b.clone()
        hs = [hvd.allreduce_async_(t, name=n, op=hvd.Sum, compression_bf16=True) for n, t in (("a", a), ("b", b))]
        for h in hs:
            hvd.synchronize(h)
        assert torch.equal(a, ra.to(torch.bfloat16).float()) and torch.equal(b, rb.to(torch.bfloat16).float())
        g = hvd.allgather(torch.ones(2, 3, device=gpu))
        assert g.shape == (2, 3)
        # DistributedOptimizer on the GPU == plain SGD at world 1
        torch.manual_seed(0)
        m = Net().to(gpu).eval()
        ref = Net().to(gpu).eval()
        ref.load_state_dict(m.state_dict())
        opt = hvd.DistributedOptimizer(torch.optim.SGD(m.parameters(), lr=0.1),
                                       named_parameters=m.named_parameters())
        xs = torch.randn(32, 1, 28, 28, device=gpu)
        ys = torch.randint(0, 10, (32,), device=gpu)
        OF.nll_loss(m(xs), ys).backward()
        opt.step()
        ropt = torch.optim.SGD(ref.parameters(), lr=0.1)
        OF.nll_loss(ref(xs), ys).backward()
        ropt.step()
        for p, q in zip(m.parameters(), ref.parameters()):
            assert torch.allclose(p, q, atol=1e-5)
    finally:
        hvd.shutdown()


_GRAPH_ALLREDUCE = r"""
import os, sys, torch, torch.distributed as dist
sys.path.insert(0, os.environ["REPO"])
from pytorch_distributed_examples_amd.parallel import dist as pdist
from pytorch_distributed_examples_amd.parallel.ddp import DistributedDataParallel
from pytorch_distributed_examples_amd.parallel.rccl import StreamComm
ctx = pdist.init_distributed()
comm = StreamComm(ctx.device)
t = torch.ones(21840, device=ctx.device)
comm.allreduce_(t, avg=True)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    for _ in range(3):   # the bench records several steps, each with its gradient all-reduce
        t.mul_(2.0)
        comm.allreduce_async(t, avg=True).wait()
g.replay()
g.replay()
torch.cuda.synchronize()
assert torch.all(t == 64.0), t[:4]
# the DDP wrapper on the plug-in (ctor broadcast of params + int64 buffers, flat-buffer all-reduce)
m = torch.nn.Sequential(torch.nn.Linear(8, 4), torch.nn.BatchNorm1d(4)).to(ctx.device)
ddp = DistributedDataParallel(m, overlap=False, comm=comm)
ddp.zero_grad()
ddp.flat_grad.fill_(3.0)
ddp.sync_gradients()
torch.cuda.synchronize()
assert torch.all(ddp.flat_grad == 3.0)
comm.destroy()
dist.destroy_process_group()
print("GRAPH_ALLREDUCE_OK")
"""


def test_stream_rccl_allreduce_inside_hipgraph(gpu):
    """bench.py records the DDP gradient all-reduce inside a hipGraph of several training steps.  c10d's
    ProcessGroupNCCL cannot be captured on this ROCm build (its watchdog aborts the process with
    hipErrorStreamCaptureUnsupported, measured), so the data plane is parallel/rccl.py's stream-ordered
    RCCL communicator: world 1 on one GPU, same call pattern, own process (own process group)."""
    import os
    import subprocess
    import sys

    from pytorch_distributed_examples_amd.parallel.dist import free_port

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, REPO=repo, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()),
               RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    env.pop("PDE_BACKEND", None)
    r = subprocess.run([sys.executable, "-c", _GRAPH_ALLREDUCE], env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0 and "GRAPH_ALLREDUCE_OK" in r.stdout, r.stderr[-3000:]


def test_hvd_aborted_communicator_raises(gpu):
    """A failed communicator surfaces as HorovodInternalError from synchronize() (what hvd.elastic.run
    catches to restore the last commit), and the engine stays failed until reset."""
    from pytorch_distributed_examples_amd import hvd
    from pytorch_distributed_examples_amd.hvd import core

    hvd.init()
    try:
        t = torch.ones(64, device=gpu)
        hvd.synchronize(hvd.allreduce_async_(t, name="before", op=hvd.Sum))
        core._ctx.comm.abort()  # what the watchdog does to a hung collective
        with pytest.raises(hvd.HorovodInternalError):
            hvd.synchronize(hvd.allreduce_async_(t, name="after", op=hvd.Sum))
        with pytest.raises(hvd.HorovodInternalError):
            hvd.allreduce_async_(t, name="later", op=hvd.Sum)
    finally:
        hvd.shutdown(abort=True)
    hvd.init()  # a fresh engine + communicator (the elastic reset path)
    try:
        t = torch.full((8,), 2.0, device=gpu)
        assert torch.equal(hvd.allreduce(t, op=hvd.Sum), t)
    finally:
        hvd.shutdown()


def test_rccl_abort_and_reinit_rounds(gpu):
    """The in-process re-wire's GPU data plane (elastic/rewire.py RoundComm) at world 1: a round's communicator
    carries stream-ordered all-reduces checked by the host-side liveness wait, is ABORTED (what a survivor does
    on a peer failure), and the next round builds a fresh communicator from a new unique id on the same device
    and keeps working -- three rounds in one process."""
    from pytorch_distributed_examples_amd import _native
    from pytorch_distributed_examples_amd.elastic.rewire import RoundComm

    C = _native.comm()

    class _Rdzv:  # no membership change published
        def hosts_updated(self):
            return False

    for rnd in range(3):
        rc = RoundComm.__new__(RoundComm)  # the round's data plane only (its gloo control plane needs peers)
        rc.rdzv, rc.rank, rc.size, rc.device = _Rdzv(), 0, 1, gpu
        rc.timeout_s, rc.grace_s, rc._steps = 30.0, 2.0, []
        rc.rccl = C.RcclComm()
        rc.rccl.init(C.rccl_unique_id(), 0, 1, gpu.index, True)
        rc.supports_avg = True
        t = torch.full((4096,), float(rnd + 1), device=gpu)
        for _ in range(3):
            rc.allreduce_async(t, avg=True)
            rc.step_done(lag=1)  # host checks the previous step's event (liveness wait)
        rc.drain()
        assert rc.rccl.async_error() in (0, 7)
        assert torch.equal(t.cpu(), torch.full((4096,), float(rnd + 1)))
        if rnd < 2:
            rc.abort()  # survivor path: abort, never destroy
            rc.rccl = None
        else:
            rc.rccl.destroy()  # (RoundComm.close would also tear down the round's gloo group)


def _clean_env():
    """The parent's env minus the rendezvous variables earlier in-process tests exported."""
    drop = ("MASTER_ADDR", "MASTER_PORT", "RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE")
    return {k: v for k, v in os.environ.items() if k not in drop and not k.startswith("TORCHELASTIC_")}


def _bench_json(out):
    import json

    lines = [ln for ln in out.splitlines() if ln.startswith('{"metric"')]
    assert lines, out[-3000:]
    return json.loads(lines[-1])


def test_hvd_cnn_bench_world1_graph(gpu):
    """``bench.py --model hvd_cnn`` at world 1: the Horovod optimizer wrapper around the fused CNN, captured."""
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--model", "hvd_cnn", "--steps", "20",
                          "--warmup", "5"], capture_output=True, text=True, timeout=300, env=_clean_env())
    assert res.returncode == 0, res.stderr[-3000:]
    rec = _bench_json(res.stdout)
    assert rec["config"]["hipgraph"] and rec["config"]["fused_step"] and rec["value"] > 1e6, rec


def test_hvd_cnn_world2_one_gpu_rehearsal(gpu):
    """Two Horovod ranks sharing the card (RCCL refuses that; the engine's xGMI one-shot data plane does
    not): the first step negotiates through the fusion engine, then graph mode reduces the flat gradient
    buffer in place, stream-ordered, inside the captured step -- no string negotiation in steady state."""
    import subprocess
    import sys

    from dist_utils import free_port

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(_clean_env(), PDE_BACKEND="gloo", PYTHONPATH=repo)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), os.path.join(repo, "bench.py"), "--gpus", "2", "--model",
           "hvd_cnn", "--steps", "20", "--warmup", "5"]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    assert res.returncode == 0, (res.stdout[-2000:], res.stderr[-3000:])
    rec = _bench_json(res.stdout)
    eng = rec["config"]["engine"]
    assert rec["n_gpus"] == 2 and rec["config"]["hipgraph"], rec
    # (inline calls are recorded once per captured step: the multi-step graph's steps + the single-step graph)
    assert eng["xgmi_batches"] >= 1 and eng["inplace_batches"] >= 1, eng
    assert eng["inline_calls"] >= rec["config"]["steps_per_graph"] + 1, (eng, rec["config"]["steps_per_graph"])
    assert eng["string_gathers"] <= 3, eng  # broadcast_parameters + the first step only
    os.makedirs(os.path.join(repo, "gpurun_out"), exist_ok=True)
    with open(os.path.join(repo, "gpurun_out", "hvd_world2_rehearsal.json"), "w") as f:
        f.write(res.stdout.strip().splitlines()[-1] + "\n")
