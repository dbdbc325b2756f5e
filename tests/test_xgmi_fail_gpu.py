"""Failure handling of the one-shot xGMI exchange (csrc/comm/xgmi_device.h), rehearsed with 2 processes on
ONE GPU (each maps the other's IPC buffer exactly as peers do over xGMI):

* a forced peer timeout sets the host-mapped error word (read without a device sync), ``check()`` raises
  and clears it, and the NEXT all-reduce is exact on both ranks (the word used to be sticky and
  silently dropped every later sum);
* the host abort word ends a spinning wait long before its timeout (elastic detection latency);
* the Horovod engine turns a timed-out exchange inside graph mode (``allreduce_inline``, no engine cycle)
  into HorovodInternalError at ``hvd.check_health()`` / ``State.commit()``.
"""
import os
import subprocess
import sys
import tempfile

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_XGMI = r"""
import os, sys, time, threading, torch, torch.distributed as dist
sys.path.insert(0, os.environ["REPO"])
from pytorch_distributed_examples_amd.parallel import dist as pdist
from pytorch_distributed_examples_amd.parallel.xgmi_allreduce import XgmiAllreduce
ctx = pdist.init_distributed()
N, r, dev = ctx.world_size, ctx.rank, ctx.device
assert N == 2
# 1. forced timeout on rank 0 (short bound), rank 1 late
xt = XgmiAllreduce(dev, max_bytes=1 << 20, timeout_s=(0.2 if r == 0 else 20.0), key="fail1")
dist.barrier()
x = torch.full((4096,), float(r + 1), device=dev)
if r == 1:
    time.sleep(1.0)
xt.allreduce_(x)
torch.cuda.synchronize()
if r == 0:
    assert xt.failed(), "timeout not reported in the host-mapped word"
    assert torch.all(x == 1.0), "a timed-out call must drop its result (local values kept)"
    try:
        xt.check()
        raise AssertionError("check() did not raise")
    except RuntimeError as e:
        assert "timed out" in str(e)
    assert not xt.failed(), "check() must clear the error words"
else:
    assert torch.all(x == 3.0), x[:4]  # the late rank still read rank 0's published chunk
    xt.check()
dist.barrier()
# 2. the next calls are exact on both ranks (no sticky fail-fast)
for k in range(3):
    y = torch.full((21840,), float(r + 1 + k), device=dev)
    xt.allreduce_(y)
    torch.cuda.synchronize()
    assert torch.all(y == float(3 + 2 * k)), (k, y[:4])
xt.check()
# 3. host abort: rank 0 spins (30 s bound) for a rank that arrives 2 s later; a host thread aborts at 0.3 s
xa = XgmiAllreduce(dev, max_bytes=1 << 20, timeout_s=30.0, key="fail2")
dist.barrier()
z = torch.full((1024,), float(r + 1), device=dev)
if r == 0:
    th = threading.Timer(0.3, xa.abort)
    t0 = time.perf_counter()
    th.start()
    xa.allreduce_(z)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    assert dt < 1.5, f"abort took {dt:.2f} s"
    assert xa.failed()
    try:
        xa.check()
        raise AssertionError("check() did not raise after abort")
    except RuntimeError:
        pass
    xa.reset_abort()
    print("ABORT_S", round(dt, 3))
else:
    time.sleep(2.0)
    xa.allreduce_(z)
    torch.cuda.synchronize()
    assert torch.all(z == 3.0)
dist.barrier()
w = torch.full((1024,), float(r + 1), device=dev)
xa.allreduce_(w)
torch.cuda.synchronize()
assert torch.all(w == 3.0), w[:4]
xa.check()
dist.barrier()
xt.close(); xa.close()
dist.destroy_process_group()
print("FAIL_OK", r)
"""

_HVD = r"""
import os, sys, time, torch
sys.path.insert(0, os.environ["REPO"])
from pytorch_distributed_examples_amd import hvd
from pytorch_distributed_examples_amd.hvd.exceptions import HorovodInternalError
os.environ["PDE_HVD_DATA_PLANE"] = "xgmi"
hvd.init()
r = hvd.rank()
dev = torch.device("cuda", torch.cuda.current_device())
g = torch.full((1000,), float(r + 1), device=dev)
hvd.allreduce_(g, op=hvd.Sum, name="g")          # negotiated once through the engine (cached)
torch.cuda.synchronize()
assert torch.all(g == 3.0)
hvd.barrier()
if r == 1:
    time.sleep(1.5)
g.fill_(float(r + 1))
try:
    hvd.core.allreduce_inline_([g], op=hvd.Sum)  # graph-mode path: no engine cycle sees this call
    torch.cuda.synchronize()
except HorovodInternalError as e:
    # the late rank: by now rank 0's engine has failed and stopped its lockstep loop, so this rank's engine
    # already saw the peer failure on the control plane (typed, never a hang)
    assert r == 1, e
    print("PEER_FAILURE_SEEN", r, str(e)[:80])
if r == 0:
    try:
        hvd.core.check_health()
        raise AssertionError("check_health did not raise")
    except HorovodInternalError as e:
        assert "xGMI" in str(e), e
    try:
        hvd.allreduce_(torch.ones(4, device=dev), name="h")
        raise AssertionError("a failed engine accepted a request")
    except HorovodInternalError:
        pass
print("HVD_FAIL_OK", r)
os._exit(0)   # the failed engine's peer state is not torn down cleanly on purpose
"""


def _run(script, env_extra):
    from pytorch_distributed_examples_amd.parallel.dist import free_port

    env = dict(os.environ, REPO=REPO, PDE_BACKEND="gloo", **env_extra)
    with tempfile.NamedTemporaryFile("w", suffix=".py", delete=False) as f:
        f.write(script)
        path = f.name
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), path]
    try:
        return subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=180)
    finally:
        os.unlink(path)


def test_xgmi_timeout_clear_and_abort(gpu):
    res = _run(_XGMI, {})
    assert res.returncode == 0 and res.stdout.count("FAIL_OK") == 2, (res.stdout[-2000:], res.stderr[-4000:])
    print([l for l in res.stdout.splitlines() if l.startswith("ABORT_S")])


def test_hvd_graph_mode_xgmi_failure_raises(gpu):
    res = _run(_HVD, {"PDE_XGMI_TIMEOUT_S": "0.3"})
    assert res.returncode == 0 and res.stdout.count("HVD_FAIL_OK") == 2, (res.stdout[-2000:], res.stderr[-4000:])
