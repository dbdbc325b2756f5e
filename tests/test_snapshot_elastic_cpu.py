"""Checkpoint format compatibility (mnist_ddp_elastic.py:95-104) and the elastic DDP
entry script under torchrun: training, snapshot resume, and restart after an injected worker failure
(torchrun --max-restarts), all on gloo."""
import os
import re

import torch

from dist_utils import REPO, torchrun
from pytorch_distributed_examples_amd.elastic.snapshot import load_snapshot, save_snapshot
from pytorch_distributed_examples_amd.models.mlp import reference_mlp

SCRIPT = os.path.join(REPO, "pytorch_elastic", "mnist_ddp_elastic.py")


def test_snapshot_roundtrip_and_reference_format(tmp_path):
    m = reference_mlp()
    p = tmp_path / "snapshot.pt"
    save_snapshot(str(p), m.state_dict(), 3, {"state": {}, "param_groups": []})
    snap = load_snapshot(str(p))
    assert snap["EPOCHS_RUN"] == 3 and set(snap) == {"MODEL_STATE", "EPOCHS_RUN", "OPTIMIZER_STATE"}
    m2 = reference_mlp()
    m2.load_state_dict(snap["MODEL_STATE"])
    assert all(torch.equal(a, b) for a, b in zip(m.state_dict().values(), m2.state_dict().values()))
    # a snapshot written exactly like the reference (plain torch.save, 2 keys) loads too
    ref = tmp_path / "ref.pt"
    torch.save({"MODEL_STATE": m.state_dict(), "EPOCHS_RUN": 1}, str(ref))
    assert load_snapshot(str(ref))["EPOCHS_RUN"] == 1
    # atomic write: no temp files left behind
    assert sorted(os.listdir(tmp_path)) == ["ref.pt", "snapshot.pt"]


def test_elastic_ddp_train_and_resume(tmp_path):
    snap = str(tmp_path / "snapshot.pt")
    args = [SCRIPT, "2", "1", "--train_size", "2048", "--test_size", "512", "--snapshot_path", snap,
            "--device", "cpu"]
    rc, out = torchrun(args, nproc=2)
    assert rc == 0, out
    assert "Local Rank: 1 | Global Rank: 1 | Epoch 1 | Batchsize: 128 | Steps: 8" in out
    assert "Training snapshot saved" in out and "Execution time" in out
    assert load_snapshot(snap)["EPOCHS_RUN"] == 1
    # resume: the saved epoch is re-run (reference semantics, Q4)
    rc, out = torchrun([SCRIPT, "3", "1", "--train_size", "2048", "--test_size", "512", "--snapshot_path", snap,
                        "--device", "cpu"], nproc=2)
    assert rc == 0, out
    assert "Resuming training from snapshot at Epoch 1" in out
    assert "Epoch 0 |" not in out.replace("Epoch 0 | Training", "")


def test_elastic_ddp_restarts_after_worker_failure(tmp_path):
    snap = str(tmp_path / "snapshot.pt")
    marker = str(tmp_path / "fault.once")
    args = ["--max-restarts", "3", SCRIPT, "2", "1", "--train_size", "2048", "--test_size", "256",
            "--snapshot_path", snap, "--device", "cpu"]
    env = {"PDE_FAULT_AT_STEP": "10", "PDE_FAULT_RANK": "1", "PDE_FAULT_MODE": "exit", "PDE_FAULT_ONCE": marker}
    rc, out = torchrun(args, nproc=2, env=env)
    assert rc == 0, out
    assert os.path.exists(marker)
    assert "[fault-injector] rank 1 step 10" in out
    # the group restarted: after the fault the job resumed from the epoch-0 snapshot and finished
    assert re.search(r"Resuming training from snapshot at Epoch 0", out), out[-3000:]


HVDRUN = ["python", "-m", "pytorch_distributed_examples_amd.launch.hvdrun"]


def test_rewire_survives_worker_failure_in_process(tmp_path):
    """--rewire: a worker dies mid-epoch; the survivor keeps its process (same pid across rounds), restores
    its in-memory commit and continues with the replacement worker -- no job restart."""
    from dist_utils import run_cmd

    env = {"PDE_FAULT_AT_STEP": "40", "PDE_FAULT_RANK": "1", "PDE_FAULT_MODE": "exit",
           "PDE_FAULT_ONCE": str(tmp_path / "once")}
    rc, out = run_cmd(HVDRUN + ["-np", "2", "--min-np", "1", "--verbose", SCRIPT, "3", "1", "--rewire", "--device",
                                "cpu", "--train_size", "8192", "--test_size", "512", "--snapshot_path",
                                str(tmp_path / "s.pt")], env=env)
    assert rc == 0, out
    assert "[fault-injector] rank 1 step 40" in out and "peer failure" in out, out[-3000:]
    pids0 = re.findall(r"\[rewire\] round 0: rank 0 of 2 \(pid (\d+)[,)]", out)
    pids1 = re.findall(r"\[rewire\] round 1: rank 0 of \d \(pid (\d+)[,)]", out)
    assert pids0 and pids1 and pids0 == pids1, out[-3000:]  # rank 0 survived in-process
    fin = re.findall(r"\[rewire\] finished 3 epochs in round (\d+)", out)
    assert len(fin) == 2 and set(fin) == {"1"}, out[-3000:]


def test_rewire_scale_up_via_discovery(tmp_path):
    """A host-discovery script that grows from 1 to 2 slots: the running worker picks the newcomer up at its
    next commit point and both finish in the same round."""
    from dist_utils import run_cmd

    snap = tmp_path / "s.pt"
    disc = tmp_path / "discover.sh"  # a second slot appears once the first epoch's snapshot exists
    disc.write_text(f"#!/bin/bash\nif [ -f {snap} ]; then echo localhost:2; else echo localhost:1; fi\n")
    disc.chmod(0o755)
    rc, out = run_cmd(HVDRUN + ["--min-np", "1", "--max-np", "2", "--host-discovery-script", str(disc), "--verbose",
                                SCRIPT, "4", "2", "--rewire", "--device", "cpu", "--train_size", "16384",
                                "--test_size", "512", "--snapshot_path", str(snap)])
    assert rc == 0, out
    assert "membership changed, re-joining" in out, out[-3000:]
    assert re.search(r"\[rewire\] round 1: rank 1 of 2", out), out[-3000:]
    fin = re.findall(r"\[rewire\] finished 4 epochs in round (\d+) \(world (\d)", out)
    assert len(fin) == 2 and all(w == "2" for _, w in fin), out[-3000:]


def test_round_shrink_plan():
    """Shrink-only re-wire: a round whose members are a subset of the previous round's, in the
    same relative order, is built by shrinking the previous RCCL communicator (excluded = the parent ranks
    that left); growth, reordering or no parent falls back to a fresh init."""
    from pytorch_distributed_examples_amd.elastic.rewire import RoundComm

    class P:  # a previous round: members in rank order, a live communicator
        def __init__(self, members):
            self.members, self.rccl = members, object()

    def plan(parent_members, members):
        rc = RoundComm.__new__(RoundComm)
        rc.members = members
        return rc._shrink_plan(P(parent_members) if parent_members is not None else None)

    assert plan(["a", "b", "c", "d"], ["a", "c", "d"]) == [1]
    assert plan(["a", "b", "c", "d"], ["b", "c"]) == [0, 3]
    assert plan(["a", "b", "c"], ["a", "b", "c", "e"]) is None      # growth: fresh init
    assert plan(["a", "b", "c"], ["a", "b", "c"]) is None           # no change
    assert plan(["a", "b", "c"], ["c", "a"]) is None                # reordered ranks
    assert plan(None, ["a"]) is None
