"""Elastic DDP benchmark (BASELINE config 2: "MNIST elastic DDP (torchrun rendezvous) scaling 2->8 MI355X
mid-run"; reference: pytorch_elastic/mnist_ddp_elastic.py:6 launched under torchrun's elastic agent).

    python bench.py --model elastic_cnn --gpus 2 --scale-to 8 [--steps K --warmup W]
    python bench.py --model elastic_cnn --gpus 2 --scale-to 1 --fault-at 300   # survive a dead worker

The parent (no GPU context) starts the elastic driver (:mod:`..launch.hvdrun`) with a host-discovery
script that reads a hosts file holding ``localhost:N``; the workers train the MNIST CNN with the fused
step + in-kernel xGMI exchange + a hipGraph per round (:func:`..elastic.rewire.run_elastic_fused`).  After
the first round's timed window, rank 0 rewrites the hosts file to ``localhost:M``: the driver spawns the
new workers and publishes a new round, the survivors notice it at their next commit point, keep their
processes, device state and data, re-wire (new control group, new xGMI peer mappings, state broadcast
from rank 0, graph recapture) and time the new world.  Output: one JSON line per round while running
(``"event": "round"``) and the bench contract's final line, whose ``value`` is the final round's
whole-node images/s and whose ``config.rounds`` lists every round with its img/s and the re-wire latency
(the slowest member's time from seeing the membership change to the first completed step of the new
round, graph capture included) with its parts (``rewire_parts``: rendezvous / control group / state
broadcast / xGMI mapping / graph capture).

``--fault-at S`` (failure rehearsal, horovod/horovod_mnist_elastic.py:55,104-106 semantics): every worker is
its own discovery "host"; the LAST rank exits at training step S of the first round (PDE_FAULT_*); the
driver blacklists its host, the survivors' in-kernel exchange times out ONCE (the error word makes every
later wait of that instance fail fast), the next commit point turns it into PeerFailure, the survivors
restore their in-memory commit and re-join at world N-1 in-process, and the new round is timed.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import tempfile
import time

METRIC = "images/sec (whole node) MNIST DDP + ResNet50 RPC-MP at 1/2/4/8 MI355X"


def parent(args, bench_py: str) -> int:
    n, m = int(args.gpus or 2), int(args.scale_to or args.gpus or 2)
    tmp = tempfile.mkdtemp(prefix="pde_elastic_")
    hosts = os.path.join(tmp, "hosts")
    fault_at = getattr(args, "fault_at", None)
    with open(hosts, "w") as f:  # fault rehearsal: one host per worker, so the blacklist drops only the dead one
        f.write("".join(f"w{i}:1\n" for i in range(n)) if fault_at is not None else f"localhost:{n}\n")
    disc = os.path.join(tmp, "discover.sh")
    with open(disc, "w") as f:
        f.write(f"#!/bin/sh\ncat {hosts}\n")
    os.chmod(disc, 0o755)
    report = os.path.join(tmp, "rounds.jsonl")
    replays = max(1, args.steps // max(1, args.graph_steps))
    cmd = [sys.executable, "-m", "pytorch_distributed_examples_amd.launch.hvdrun", "--host-discovery-script", disc,
           "--min-np", str(min(n, m)), "--max-np", str(max(n, m)), "--discovery-interval", "0.5",
           *(["--blacklist-cooldown-range", "3600", "3600"] if fault_at is not None else []), bench_py,
           "--model", "elastic_cnn", "--elastic-worker", "--scale-to", str(m), "--hosts-file", hosts,
           "--report", report, "--steps", str(args.steps), "--warmup", str(args.warmup),
           "--graph-steps", str(args.graph_steps), "--batch", str(args.batch or 1024), "--device", args.device,
           *(["--fault-at", str(fault_at)] if fault_at is not None else [])]
    env = dict(os.environ)
    if fault_at is not None:
        env.update(PDE_FAULT_AT_STEP=str(fault_at), PDE_FAULT_RANK=str(n - 1), PDE_FAULT_MODE="exit",
                   PDE_FAULT_ONCE=os.path.join(tmp, "fault.once"))
    env.setdefault("OMP_NUM_THREADS", "1")
    repo = os.path.dirname(os.path.abspath(bench_py))
    env["PYTHONPATH"] = repo + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    t0 = time.time()
    rc = subprocess.call(cmd, env=env, timeout=float(os.environ.get("PDE_ELASTIC_BENCH_TIMEOUT", "900")))
    rounds = []
    if os.path.exists(report):
        with open(report) as f:
            rounds = [json.loads(line) for line in f if line.strip()]
    if rc != 0 or not rounds:
        print(json.dumps({"error": f"elastic bench failed rc={rc}", "rounds": rounds}), flush=True)
        return rc or 1
    last = rounds[-1]
    gpu = args.device != "cpu"
    print(json.dumps({
        "metric": METRIC, "value": round(last["images_per_s"], 1), "unit": "images/s", "n_gpus": last["world"],
        "steps": replays * args.graph_steps, "warmup": args.warmup, "ms_per_step": round(last["ms_per_step"], 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16" if args.device != "cpu" else "fp32",
        "data": "synthetic (random init)",
        "config": {"model": "mnist_cnn_Net", "baseline_config": "2: MNIST elastic DDP scaling mid-run",
                   "global_batch": (args.batch or 1024) * last["world"], "seq_len": None, "image": "1x28x28",
                   "parallelism": f"dp{n}->dp{m} (in-process re-wire{', worker killed' if fault_at is not None else ''})", "fused_step": gpu, "hipgraph": gpu,
                   "allreduce": "xgmi-in-reduce-kernel" if gpu else "gloo", "rounds": rounds,
                   "wall_s": round(time.time() - t0, 2)},
    }), flush=True)
    return 0


def worker(args) -> None:
    """One elastic worker (launched by the driver)."""
    from ..elastic.rewire import run_elastic_fused

    n_target = int(args.scale_to)
    fault_mode = getattr(args, "fault_at", None) is not None
    requested = [False]

    def report(rnd, rank, size, info):
        if rank == 0:
            rec = dict(event="round", round=rnd, world=size, **{k: (round(v, 4) if isinstance(v, float) else v)
                                                                for k, v in info.items()})
            sys.stdout.write(json.dumps(rec) + "\n")  # ONE write: other ranks' log lines never split the record
            sys.stdout.flush()
            with open(args.report, "a") as f:
                f.write(json.dumps(rec) + "\n")
            if size != n_target and not requested[0] and not fault_mode:  # the discovery script reads this file
                with open(args.hosts_file, "w") as f:
                    f.write(f"localhost:{n_target}\n")
                requested[0] = True
        if fault_mode:  # keep training into the injected fault; finish once the survivors' round is measured
            return rnd > 0 and size == n_target
        return size == n_target  # the target world has been measured: finish

    class A:
        pass

    a = A()
    a.batch_size = args.batch or 1024
    a.graph_steps = args.graph_steps
    a.commit_every = 10  # replays between commit points (device-side commits: no sync, rewire.py _DeviceCommit)
    a.round_warmup = max(1, args.warmup // max(1, args.graph_steps))
    a.round_replays = max(1, args.steps // max(1, args.graph_steps))
    a.total_steps = 10 ** 9  # the bench ends through report()
    a.total_epochs = 10 ** 6
    a.train_size = 60000  # the reference's MNIST train set (HBM-resident synthetic samples) ...
    a.test_size = 10000
    # ... over a longer virtual epoch, so every round's timed window fits in whole replays of one epoch
    a.virtual_train_size = max(60000, (a.round_warmup + a.round_replays + 2) * a.graph_steps * a.batch_size *
                               max(n_target, int(args.gpus or 2)))
    a.save_every = 0
    a.device = args.device
    run_elastic_fused(a, report=report)
