"""Pipeline data plane over xGMI (csrc/comm/p2p_ring.hip) rehearsed on ONE GPU: two processes share the card
and write into each other's IPC-mapped receive rings exactly as two stage GPUs of a node do over their direct
xGMI link.

* the raw channel: messages of many sizes (1 B .. 3 slots) in both directions, more messages in flight than
  ring slots (credits), a late receiver, and send/recv captured into a hipGraph and replayed;
* BASELINE config 3's step: the 2-stage ResNet-50 (``ResNetPipelineDP``, gpipe and 1f1b) captured into ONE
  hipGraph per rank -- micro-batch forwards/backwards, ring sends on the side stream, ring receives, SGD --
  against a single-process run of the same shards on the same batch: losses and final weights must agree;
* the RPC form (``RemotePipeline`` / ``resnet_rpc``): master + 2 stage workers, stage activations over the ring.
The world-N versions on real GPUs are in tests/test_multigpu.py."""
import os
import subprocess
import sys
import tempfile
import time

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_RING = r"""
import os, sys, time, torch, torch.distributed as dist
sys.path.insert(0, os.environ["REPO"])
from pytorch_distributed_examples_amd.parallel import dist as pdist
from pytorch_distributed_examples_amd.parallel.pipeline import P2PChannel
ctx = pdist.init_distributed()          # PDE_BACKEND=gloo: two ranks on one GPU
r, dev = ctx.rank, ctx.device
os.environ["PDE_P2P_SLOT_MB"] = "0.25"  # 256 KB slots: large tensors span several messages
ch = P2PChannel(1 - r, "ringtest", dev)
assert ch.mode == "ring" and ch.ring is not None

def data(k, n, dtype):
    g = torch.Generator().manual_seed(7 * k + n)
    return (torch.randn(n, generator=g) * 100).to(dtype)

sizes = [(1, torch.uint8), (7, torch.bfloat16), (1000, torch.float32), (65536, torch.bfloat16),
         (3 * 65536 + 5, torch.float32), (123457, torch.bfloat16), (16, torch.int64)] * 3
# rank 0 streams everything down while rank 1 streams everything up (both directions at once, > 4 slots
# in flight per direction: the senders wait on credits), then each receives and checks
if r == 1:
    time.sleep(0.5)  # a late receiver: rank 0's sends wait for credits, bounded
for k, (n, dt) in enumerate(sizes):
    ch.send(data(k + 100 * r, n, dt).to(dev))
got = [ch.recv((n,), dt) for n, dt in sizes]
ch.flush()
torch.cuda.synchronize()
ch.check()
for k, ((n, dt), t) in enumerate(zip(sizes, got)):
    assert torch.equal(t.cpu(), data(k + 100 * (1 - r), n, dt)), (r, k, n, dt)
# hipGraph: one captured exchange (send then recv), replayed 5 times with new payloads
src = torch.zeros(50000, device=dev)
torch.cuda.synchronize()
dist.barrier()
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    with torch.cuda.graph(g):
        ch.send(src)
        out = ch.recv((50000,), torch.float32)
        ch.flush()
for it in range(5):
    src.fill_(float(10 * it + r))
    g.replay()
    torch.cuda.synchronize()
    assert torch.all(out == float(10 * it + 1 - r)), (it, out[:3])
ch.check()
dist.barrier()
ch.close()
dist.destroy_process_group()
print("RING_OK", r)
"""

_PIPE = r"""
import os, sys, torch, torch.distributed as dist
sys.path.insert(0, os.environ["REPO"])
from pytorch_distributed_examples_amd.parallel import dist as pdist
from pytorch_distributed_examples_amd.apps.hybrid_ps import ResNetPipelineDP
from pytorch_distributed_examples_amd.utils.graph import CapturedStep
schedule = os.environ["SCHEDULE"]
ctx = pdist.init_distributed()          # PDE_BACKEND=gloo: the pipeline's two stages on one GPU
r, dev = ctx.rank, ctx.device
B, M, IMG, STEPS = 8, 2, 64, 3
torch.manual_seed(0)
pipe = ResNetPipelineDP(ctx, batch=B, split_size=M, image=IMG, schedule=schedule, lr=0.05)
assert pipe.mb_group == int(os.environ["PDE_PIPE_MB_GROUP"]), pipe.mb_group
assert pipe.capturable, "ring data plane + dp1: the whole step must be capturable"
graph = CapturedStep(pipe.step, [], warmup=1).capture()   # one eager warm-up step (meta handshake), then capture
losses = [float(graph().item()) for _ in range(STEPS)]
pipe.check()
flat = torch.cat([p.detach().float().reshape(-1) for p in pipe.module.parameters()]).cpu()
# reference: the same two shards, same init, same batch, in ONE process (rank 0), same micro-batching (the
# grouped-vs-separate BatchNorm equivalence itself: test_batchnorm_groups / test_resnet_pipeline_mb_groups_match)
objs = [None, None]
dist.all_gather_object(objs, (losses, flat))
if r == 0:
    from pytorch_distributed_examples_amd.data.synthetic import resnet_batch
    from pytorch_distributed_examples_amd.models.resnet import ResNetShard1, ResNetShard2
    from pytorch_distributed_examples_amd.ops import functional as OF
    from pytorch_distributed_examples_amd.ops.optim import FusedSGD
    torch.manual_seed(0); s1 = ResNetShard1().to(dev)
    torch.manual_seed(0); s2 = ResNetShard2().to(dev)
    g = torch.Generator().manual_seed(1234)
    x, y = resnet_batch(B, IMG, 1000, dev, g)
    opt = FusedSGD(list(s1.parameters()) + list(s2.parameters()), lr=0.05)
    ref_losses = []
    for step in range(1 + STEPS):    # the warm-up step + the timed replays
        for p in list(s1.parameters()) + list(s2.parameters()):
            p.grad = None
        tot = 0.0
        G = pipe.mb_group  # same units, same grouped BatchNorm: identical numerics to the pipelined step
        for xm, ym in zip(x.split(M * G), y.split(M * G)):
            with OF.bn_groups(G):
                loss = OF.mse_loss(s2(s1(xm)), ym) / (B // (M * G))
            loss.backward()
            tot += float(loss.item())
        opt.step()
        ref_losses.append(tot)
    pl = objs[1][0]
    assert all(abs(a - b) <= 2e-3 * max(1.0, abs(b)) for a, b in zip(pl, ref_losses[1:])), (pl, ref_losses)
    for k, mod in ((0, s1), (1, s2)):
        ref = torch.cat([p.detach().float().reshape(-1) for p in mod.parameters()]).cpu()
        err = ((objs[k][1] - ref).norm() / ref.norm()).item()
        assert err < 2e-3, (k, err)
dist.barrier()
pipe.close()
dist.destroy_process_group()
print("PIPE_OK", r)
"""


_PIPE_DP = r"""
import os, sys, json, time, torch, torch.distributed as dist
sys.path.insert(0, os.environ["REPO"])
from pytorch_distributed_examples_amd.parallel import dist as pdist
from pytorch_distributed_examples_amd.apps.hybrid_ps import ResNetPipelineDP
from pytorch_distributed_examples_amd.utils.graph import CapturedStep
ctx = pdist.init_distributed()          # PDE_BACKEND=gloo: 4 ranks = 2 pipelines x 2 stages on ONE GPU
r, dev, W = ctx.rank, ctx.device, ctx.world_size
B, M, IMG, STEPS = 8, 2, 64, 3
torch.manual_seed(0)
pipe = ResNetPipelineDP(ctx, batch=B, split_size=M, image=IMG, schedule="1f1b", lr=0.05)
if os.environ.get("PDE_PIPE_DP_COMM") != "gloo":
    assert pipe.dp == 2 and pipe.comm is not None and pipe.capturable, "xGMI DP communicator: capturable step"
SAME = os.environ.get("PIPE_DP_SAME_BATCH") == "1"  # diagnostic: both pipelines train on pipeline 0's batch
if SAME:
    from pytorch_distributed_examples_amd.data.synthetic import resnet_batch as _rb
    _x, _y = _rb(B, IMG, 1000, dev, torch.Generator().manual_seed(1234))
    _u = M * pipe.mb_group
    pipe.xs, pipe.ys = list(_x.split(_u)), list(_y.split(_u))
if os.environ.get("PIPE_DP_EAGER") == "1":  # the same split step without graphs (diagnostic A/B)
    def graph():
        pipe.ddp.zero_grad()
        loss = pipe.engine.train_step(pipe.xs if pipe.stage == 0 else None, pipe.ys if pipe.last else None, pipe.n_mb)
        torch.cuda.synchronize(); dist.barrier()
        pipe.ddp.sync_gradients(); pipe.opt.step()
        torch.cuda.synchronize(); dist.barrier()
        return loss if loss is not None else torch.zeros((), device=dev)
    graph()                       # the warm-up step
else:
    graph = pipe.split_step_graphs()  # one eager warm-up step, then 2 hipGraphs per step with a host barrier between
torch.cuda.synchronize()
t0 = time.perf_counter()
losses = [float(graph().item()) for _ in range(STEPS)]
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / STEPS
pipe.check()
if pipe.comm is not None:
    pipe.comm.check()
flat = torch.cat([p.detach().float().reshape(-1) for p in pipe.module.parameters()]).cpu()
objs = [None] * W
dist.all_gather_object(objs, (losses, flat, dict(pipe.comm.routed) if pipe.comm is not None else {}))
# the DP replicas of each stage hold bit-identical weights
assert torch.equal(objs[0][1], objs[2][1]) and torch.equal(objs[1][1], objs[3][1])
if r == 0:
    from pytorch_distributed_examples_amd.data.synthetic import resnet_batch
    from pytorch_distributed_examples_amd.models.resnet import ResNetShard1, ResNetShard2
    from pytorch_distributed_examples_amd.ops import functional as OF
    from pytorch_distributed_examples_amd.ops.optim import FusedSGD
    # one process, one model copy PER PIPELINE (each copy's modules see only their own pipeline's batches, as each
    # replica does; per-module state such as BatchNorm running statistics evolves the same way), the DP average of
    # the two copies' gradients applied to both copies with the same SGD
    copies = []
    for p in range(2):
        torch.manual_seed(0); a1 = ResNetShard1().to(dev)
        torch.manual_seed(0); a2 = ResNetShard2().to(dev)
        copies.append((a1, a2, FusedSGD(list(a1.parameters()) + list(a2.parameters()), lr=0.05)))
    s1, s2 = copies[0][0], copies[0][1]
    batches = [resnet_batch(B, IMG, 1000, dev, torch.Generator().manual_seed(1234 + (0 if SAME else p)))
               for p in range(2)]
    G = pipe.mb_group
    ref = []
    for step in range(1 + STEPS):
        per = []
        for (a1, a2, _), (x, y) in zip(copies, batches):
            for q in list(a1.parameters()) + list(a2.parameters()):
                q.grad = None
            tot = 0.0
            for xm, ym in zip(x.split(M * G), y.split(M * G)):
                with OF.bn_groups(G):
                    loss = OF.mse_loss(a2(a1(xm)), ym) / (B // (M * G))
                loss.backward()
                tot += float(loss.item())
            per.append(tot)
        pa = [q for q in list(copies[0][0].parameters()) + list(copies[0][1].parameters())]
        pb = [q for q in list(copies[1][0].parameters()) + list(copies[1][1].parameters())]
        with torch.no_grad():
            for qa, qb in zip(pa, pb):    # DDP's average (fp32, rank order)
                avg = (qa.grad + qb.grad) * 0.5
                qa.grad.copy_(avg); qb.grad.copy_(avg)
        for _, _, o in copies:
            o.step()
        ref.append(per)
    print("PIPEDP losses", [objs[1][0], objs[3][0]], "ref", ref[1:], flush=True)
    for p in range(2):  # pipeline p's loss is reported by its last stage, rank 2p + 1
        pl = objs[2 * p + 1][0]
        assert all(abs(a - b[p]) <= 2e-3 * max(1.0, abs(b[p])) for a, b in zip(pl, ref[1:])), (p, pl, ref)
    for k, mod in ((0, s1), (1, s2)):
        want = torch.cat([q.detach().float().reshape(-1) for q in mod.parameters()]).cpu()
        err = ((objs[k][1] - want).norm() / want.norm()).item()
        assert err < 3e-3, (k, err)
    rec = dict(config="4 rehearsal: resnet50 pp2 x dp2, 4 ranks sharing ONE MI355X",
               hipgraph=os.environ.get("PIPE_DP_EAGER") != "1",
               graphs_per_step="2 (pipeline part | host barrier | DP all-reduce + SGD: shared-GPU rehearsal only)",
               dp_comm="xgmi one-shot + two-shot (no RCCL), fp32 wire", loss_ref=[r for r in ref[1:]], batch_per_pipeline=B, split_size=M, image=IMG,
               mb_group=G, schedule="1f1b", steps=STEPS, ms_per_step_shared_gpu=round(dt * 1e3, 3),
               losses=[objs[1][0], objs[3][0]], routed=[o[2] for o in objs],
               note="4 processes time-share one GPU: a correctness rehearsal, not a throughput number")
    os.makedirs(os.path.join(os.environ["REPO"], "gpurun_out"), exist_ok=True)
    name = "r6_world4_shared_gpu_resnet50_pp" + ("_eager" if os.environ.get("PIPE_DP_EAGER") == "1" else "")
    with open(os.path.join(os.environ["REPO"], "gpurun_out", name + ".jsonl"), "w") as f:
        f.write(json.dumps(rec) + "\n")
dist.barrier()
pipe.close()
dist.destroy_process_group()
print("PIPEDP_OK", r)
"""


def _torchrun(script, n, extra_env=None, timeout=600):
    from pytorch_distributed_examples_amd.parallel.dist import free_port

    env = dict(os.environ, REPO=REPO, PDE_BACKEND="gloo", **(extra_env or {}))
    with tempfile.NamedTemporaryFile("w", suffix=".py", delete=False) as f:
        f.write(script)
        path = f.name
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), path]
    try:
        return subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
    finally:
        os.unlink(path)


def _check(res, tag, n, name):
    if res.returncode != 0:
        os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
        with open(os.path.join(REPO, "gpurun_out", f"{name}.err"), "w") as f:
            f.write(res.stdout + "\n----\n" + res.stderr)
    ranks = "\n".join(l for l in res.stderr.splitlines() if l.startswith("[rank"))
    assert res.returncode == 0 and res.stdout.count(tag) == n, (res.stdout[-2000:], ranks[-6000:])


def test_p2p_ring_rehearsal_one_gpu(gpu):
    _check(_torchrun(_RING, 2), "RING_OK", 2, "p2p_ring")


@pytest.mark.parametrize("schedule,group", [("gpipe", "1"), ("1f1b", "1"), ("gpipe", "4"), ("1f1b", "2")])
def test_resnet_pipeline_graph_rehearsal_one_gpu(gpu, schedule, group):
    """group = micro-batches per pipeline unit (grouped BatchNorm, PDE_PIPE_MB_GROUP); the single-process
    reference always runs one micro-batch at a time."""
    _check(_torchrun(_PIPE, 2, {"SCHEDULE": schedule, "PDE_PIPE_MB_GROUP": group}), "PIPE_OK", 2,
           f"pipe_{schedule}_g{group}")


@pytest.mark.parametrize("mode", ["graph", "eager"])
def test_resnet_pipeline_x_dp_xgmi_graph_rehearsal_one_gpu(gpu, mode):
    """BASELINE config 4's step, pp2 x dp2 = 4 ranks on one GPU: stage activations over the P2P rings, each stage's
    gradients all-reduced across its 2 replicas by the xGMI one-/two-shot communicator inside the captured step;
    losses and final weights against ONE process running both pipelines' micro-batches with averaged gradients."""
    # fp32 gradients on the DP wire: the single-process reference accumulates fp32 gradients (the bf16 wire is the
    # default elsewhere and rounds the averaged gradient: ~1 % loss drift after 3 steps at lr 0.05)
    res = _torchrun(_PIPE_DP, 4, {"PDE_PIPE_MB_GROUP": "2", "PDE_PIPE_GRAD_DTYPE": "fp32",
                                  "PIPE_DP_EAGER": "1" if mode == "eager" else "0"})
    print([l for l in res.stdout.splitlines() if l.startswith("PIPEDP losses")])
    _check(res, "PIPEDP_OK", 4, f"pipe_dp_xgmi_{mode}")


def test_resnet_rpc_pipeline_one_gpu(gpu):
    """rpc/model_parallel_ResNet50.py end to end on one GPU: master + 2 stage workers (both stages on
    cuda:0), stage activations / gradients over the P2P ring, distributed autograd + optimizer."""
    env = dict(os.environ, PDE_BACKEND="gloo")
    cmd = [sys.executable, os.path.join(REPO, "rpc", "model_parallel_ResNet50.py"), "--splits", "4",
           "--num-batches", "3", "--batch-size", "8", "--image-w", "64", "--image-h", "64", "--verbose"]
    res = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert res.returncode == 0, (res.stdout[-3000:], res.stderr[-3000:])
    assert "number of splits = 4, execution time" in res.stdout and "batch 2: loss" in res.stdout, res.stdout


_PS = r"""
import faulthandler, os, sys, torch, torch.distributed.rpc as rpc
faulthandler.dump_traceback_later(200, exit=True)  # a hang dumps every thread's stack and exits
sys.path.insert(0, os.environ["REPO"])
from torch import nn
from pytorch_distributed_examples_amd.ops import layers as L
from pytorch_distributed_examples_amd.rpc import DistributedOptimizer, RemoteModule, dist_autograd


def _table(srv):  # runs on the owner: a host copy of its table (test reference only)
    return srv.local_value().module.weight.detach().float().cpu()


rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
opts = rpc.TensorPipeRpcBackendOptions(num_worker_threads=8, rpc_timeout=120,
                                       init_method=f"tcp://127.0.0.1:{os.environ['RPC_PORT']}")
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
if rank == 0:
    rpc.init_rpc("trainer0", rank=0, world_size=world, rpc_backend_options=opts)
    emb = RemoteModule("ps/cuda:0", L.EmbeddingBag, args=(10, 3), kwargs={"mode": "sum"})
    assert emb.uses_ring(dev)
    popt = DistributedOptimizer(torch.optim.SGD, emb.remote_parameters(), lr=1.0)
    idx, off = torch.tensor([1, 2, 3, 4]), torch.tensor([0, 2])
    outs = []
    print("setup done", flush=True)
    for it in range(3):  # several steps: the ring's sequence numbers advance in both directions
        print("step", it, flush=True)
        with dist_autograd.context() as cid:
            e = emb(idx, off, out_device=dev)
            assert e.is_cuda and e.device == dev   # rows arrived in this GPU's HBM
            dist_autograd.backward(cid, [e.sum()])
            popt.step(cid)
        outs.append(e.detach().clone())
    for a, b in zip(outs, outs[1:]):
        assert torch.allclose(b, a - 2.0, atol=1e-5), (a, b)  # each looked-up row moved by -lr * 1 per step
    # a big lookup that spans several ring slots: the owner's EmbeddingBag against a host copy of its table
    big = RemoteModule("ps/cuda:0", L.EmbeddingBag, args=(5000, 256), kwargs={"mode": "sum"})
    g = torch.Generator().manual_seed(0)
    bidx = torch.randint(0, 5000, (40000,), generator=g)
    boff = torch.arange(0, 40000, 8)
    with dist_autograd.context() as cid:
        e = big(bidx, boff, out_device=dev)
    w = rpc.rpc_sync("ps", _table, args=(big.server,))
    ref = torch.nn.functional.embedding_bag(bidx, w, boff, mode="sum")
    assert torch.allclose(e.cpu(), ref, rtol=1e-4, atol=1e-4)
    emb.close()
    big.close()
    print("PS_OK", flush=True)
else:
    rpc.init_rpc("ps", rank=1, world_size=world, rpc_backend_options=opts)
rpc.shutdown()
"""


def test_parameter_server_ring_data_plane_one_gpu(gpu):
    """P6 over xGMI: a trainer process and the "ps" process share the GPU; lookups and output gradients
    move over the P2P ring (RPC carries only the call and the host indices); Hogwild SGD on the owner."""
    from pytorch_distributed_examples_amd.parallel.dist import free_port

    env = dict(os.environ, REPO=REPO, RPC_PORT=str(free_port()), PYTHONUNBUFFERED="1")
    logdir = os.path.join(REPO, "gpurun_out")
    os.makedirs(logdir, exist_ok=True)
    with tempfile.NamedTemporaryFile("w", suffix=".py", delete=False) as f:
        f.write(_PS)
        path = f.name
    logs = [os.path.join(logdir, f"ps_ring_rank{r}.log") for r in range(2)]
    try:
        files = [open(lg, "w") for lg in logs]  # progress lands under gpurun_out/ while it runs
        procs = [subprocess.Popen([sys.executable, path], env=dict(env, RANK=str(r), WORLD_SIZE="2"),
                                  stdout=fo, stderr=subprocess.STDOUT, text=True) for r, fo in enumerate(files)]
        t0 = time.time()
        while any(p.poll() is None for p in procs) and time.time() - t0 < 150:
            if any(p.poll() not in (None, 0) for p in procs):  # one side failed: the other would wait forever
                break
            time.sleep(0.5)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        for fo in files:
            fo.close()
        os.unlink(path)
    outs = [open(lg).read() for lg in logs]
    assert all(p.returncode == 0 for p in procs) and "PS_OK" in outs[0], [o[-3000:] for o in outs]


def test_hybrid_ps_script_ring_one_gpu(gpu):
    """rpc/server_model_data_parallel.py on one GPU: 2 trainers + master + ps, trainers' DDP on gloo (two
    ranks on one device), embedding rows and gradients over the P2P ring."""
    env = dict(os.environ, PDE_BACKEND="gloo", PYTHONUNBUFFERED="1")
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    log = os.path.join(REPO, "gpurun_out", "hybrid_ps_ring.log")
    with open(log, "w") as fo:  # progress lands under gpurun_out/ while it runs
        rc = subprocess.call([sys.executable, os.path.join(REPO, "rpc", "server_model_data_parallel.py"), "--epochs",
                              "6"], env=env, stdout=fo, stderr=subprocess.STDOUT, timeout=600)
    out = open(log).read()
    assert rc == 0, out[-4000:]
    assert "Training done for epoch 5" in out and "embedding data plane: p2p-ring" in out, out[-4000:]
