#!/usr/bin/env python3
"""Headline benchmark: images/sec for the whole node (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--model cnn|mlp|resnet50|resnet50_pp]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Default workload = BASELINE.json configs[1] (MNIST CNN DDP bf16, RCCL all-reduce over xGMI); see
``pytorch_distributed_examples_amd/bench/harness.py`` for every workload and the timing rules.

``--gpus N`` with N > 1 and no torchrun environment: this process launches the N ranks itself (torchrun on
127.0.0.1, one rank per GPU) WITHOUT touching the GPU first, passes its own arguments through and exits with
their status.  Under torchrun the world size must equal ``--gpus`` (checked by the harness).
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys

REPO = os.path.dirname(os.path.abspath(__file__))


def _requested_gpus(argv) -> int:
    for i, a in enumerate(argv):
        if a == "--gpus" and i + 1 < len(argv):
            return int(argv[i + 1])
        if a.startswith("--gpus="):
            return int(a.split("=", 1)[1])
    return 1


def _launch_ranks(n: int, argv) -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]
    env = dict(os.environ, OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "1"))
    return subprocess.call(cmd, env=env)


def main() -> None:
    argv = sys.argv[1:]
    n = _requested_gpus(argv)
    elastic = "elastic_cnn" in argv  # its own launcher (the elastic driver), never torchrun
    if n > 1 and "WORLD_SIZE" not in os.environ and not elastic:
        # parent: no torch import, no GPU context -- the ranks own the GPUs
        sys.exit(_launch_ranks(n, argv))
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    if REPO not in sys.path:
        sys.path.insert(0, REPO)
    from pytorch_distributed_examples_amd.bench import harness

    harness.main(argv)


if __name__ == "__main__":
    main()
