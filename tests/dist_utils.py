"""Helpers for multi-process CPU tests (gloo on 127.0.0.1, the reference's own single-host technique,
SURVEY.md §4)."""
import os
import socket
import subprocess
import sys

import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


_HANDED_OUT = set()


def free_port():
    """A free port not handed out before by this process (two quick calls can otherwise return the same one)."""
    for _ in range(64):
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        if port not in _HANDED_OUT:
            _HANDED_OUT.add(port)
            return port
    return port


def _entry(rank, world, port, fn, args):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank)})
    import torch

    torch.set_num_threads(1)
    fn(rank, world, *args)


def spawn(fn, world=2, args=()):
    """Run ``fn(rank, world, *args)`` in ``world`` processes with the env:// rendezvous set up."""
    mp.spawn(_entry, args=(world, free_port(), fn, args), nprocs=world, join=True)


def run_cmd(cmd, timeout=600, env=None):
    e = dict(os.environ)
    e["PYTHONPATH"] = REPO + os.pathsep + e.get("PYTHONPATH", "")
    e.setdefault("OMP_NUM_THREADS", "2")
    if env:
        e.update(env)
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=e, cwd="/tmp")
    return res.returncode, res.stdout + res.stderr


def torchrun(script_args, nproc=2, timeout=600, env=None):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr", "127.0.0.1", "--nproc-per-node", str(nproc)]
    return run_cmd(cmd + script_args, timeout, env)
