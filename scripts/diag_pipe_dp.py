"""Diagnostic: pp2 x dp2 ResNet pipeline on ONE GPU (4 ranks, PDE_BACKEND=gloo) with the xGMI DP communicator,
EAGER steps with a device sync + timestamped print after every phase, to locate a cross-rank wait that does not
complete.  torchrun --nproc-per-node 4 scripts/diag_pipe_dp.py [gpipe|1f1b] [graph]"""
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_examples_amd.apps.hybrid_ps import ResNetPipelineDP  # noqa: E402
from pytorch_distributed_examples_amd.parallel import dist as pdist  # noqa: E402

t0 = time.time()
ctx = pdist.init_distributed()
r = ctx.rank


def say(msg):
    print(f"[{time.time() - t0:7.2f}s r{r}] {msg}", flush=True)


sched = sys.argv[1] if len(sys.argv) > 1 else "1f1b"
torch.manual_seed(0)
pipe = ResNetPipelineDP(ctx, batch=8, split_size=2, image=64, schedule=sched, lr=0.05)
say(f"built: dp={pipe.dp} stage={pipe.stage} comm={type(pipe.comm).__name__} capturable={pipe.capturable}")
for step in range(2):
    pipe.ddp.zero_grad()
    loss = pipe.engine.train_step(pipe.xs if pipe.stage == 0 else None, pipe.ys if pipe.last else None, pipe.n_mb)
    torch.cuda.synchronize()
    say(f"step {step}: pipeline done")
    pipe.ddp.sync_gradients()
    torch.cuda.synchronize()
    say(f"step {step}: dp reduce done routed={pipe.comm.routed}")
    pipe.opt.step()
    torch.cuda.synchronize()
    pipe.check()
    pipe.comm.check()
    say(f"step {step}: ok loss={float(loss) if loss is not None else None}")
if len(sys.argv) > 2 and sys.argv[2] == "graph":
    from pytorch_distributed_examples_amd.utils.graph import CapturedStep

    g = CapturedStep(pipe.step, [], warmup=0).capture()
    say("captured")
    for i in range(3):
        g()
        torch.cuda.synchronize()
        say(f"replay {i} done")
    pipe.check()
    pipe.comm.check()
dist.barrier()
pipe.close()
say("DIAG_OK")
