"""BASELINE config 2 rehearsed on ONE GPU: the elastic bench scales 1 -> 2 workers mid-run on the fused CNN
path (whole-step kernel + gradient exchange over xGMI inside the reduction kernel, one hipGraph per round,
recaptured after the re-wire).  The two workers share the card and map each other's IPC staging buffers
exactly as two GPUs of a node do.  (3+ processes cannot rehearse this on one card: spinning exchange
workgroups of the ranks already in their reduction kernel keep a late rank's 122 KB-LDS training kernel from
being placed -- on a node every rank owns its GPU.)"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))



def _rec(line):
    """The JSON record at the start of a line (another rank's log text may follow it on the same line)."""
    return json.JSONDecoder().raw_decode(line)[0]

def test_elastic_bench_scale_up_one_gpu(gpu):
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--model", "elastic_cnn", "--gpus", "1", "--scale-to", "2",
           "--steps", "100", "--warmup", "20", "--graph-steps", "10"]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert res.returncode == 0, (res.stdout[-3000:], res.stderr[-3000:])
    rounds = [_rec(ln) for ln in res.stdout.splitlines() if ln.startswith('{"event": "round"')]
    final = [_rec(ln) for ln in res.stdout.splitlines() if ln.startswith('{"metric"')]
    assert [r["world"] for r in rounds] == [1, 2] and len(final) == 1, res.stdout[-3000:]
    assert rounds[1]["rewire_s"] is not None and rounds[1]["rewire_s"] > 0
    assert all(r["images_per_s"] > 1e6 for r in rounds), rounds  # fused path (millions of images/s)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "elastic_rehearsal.jsonl"), "w") as f:
        for r in rounds + final:
            f.write(json.dumps(r) + "\n")


def test_elastic_bench_survives_killed_worker_one_gpu(gpu):
    """BASELINE config 2 failure path on the fused / in-kernel xGMI data plane (VERDICT r3 ask 3): two workers
    share the card, rank 1 exits at step 300 of round 0; the survivor's exchange times out ONCE (error word,
    later waits fail fast), its next commit point raises PeerFailure, it restores its in-memory commit and
    re-joins at world 1 in the same process; the new round is timed and the re-wire latency is broken down."""
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--model", "elastic_cnn", "--gpus", "2", "--scale-to", "1",
           "--fault-at", "300", "--steps", "100", "--warmup", "20", "--graph-steps", "10"]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert res.returncode == 0, (res.stdout[-3000:], res.stderr[-3000:])
    out = res.stdout + res.stderr
    rounds = [_rec(ln) for ln in res.stdout.splitlines() if ln.startswith('{"event": "round"')]
    final = [_rec(ln) for ln in res.stdout.splitlines() if ln.startswith('{"metric"')]
    assert "[fault-injector] rank 1 step 300" in out and "peer failure" in out, out[-3000:]
    assert [r["world"] for r in rounds] == [2, 1] and len(final) == 1, out[-3000:]
    assert rounds[1]["rewire_s"] is not None and rounds[1]["rewire_s"] > 0
    assert set(rounds[1]["rewire_parts"]) == {"rendezvous_s", "control_s", "broadcast_s", "map_s", "capture_s",
                                              "detect_s"}
    # detection (fault -> PeerFailure): the driver's failure report raises the exchange's host abort word, so the
    # survivor does not wait out the exchange timeout (VERDICT r4 ask 4: <= 1 s)
    assert rounds[1]["rewire_parts"]["detect_s"] <= 1.0, rounds[1]
    assert all(r["images_per_s"] > 1e6 for r in rounds), rounds  # fused path
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "elastic_fault_rehearsal.jsonl"), "w") as f:
        for r in rounds + final:
            f.write(json.dumps(r) + "\n")


def test_hvd_elastic_script_survives_killed_worker_one_gpu(gpu, tmp_path):
    """horovod/horovod_mnist_elastic.py on the GPU (VERDICT r4 ask 5): two workers share the card, the step is the
    fused CNN kernel + the fusion engine's in-place xGMI all-reduce + AdamW in a hipGraph; rank 1 is killed
    mid-epoch; the survivor's engine raises HorovodInternalError (typed at the source), ``hvd.elastic.run``
    restores the last commit, resets in-process (new round, new engine), runs ``on_state_reset`` (LR =
    0.01 / sqrt(world)) and finishes; every finishing worker reports the same test accuracy."""
    env = dict(os.environ, PDE_FAULT_AT_STEP="40", PDE_FAULT_RANK="1", PDE_FAULT_MODE="exit",
               PDE_FAULT_ONCE=str(tmp_path / "once"), PDE_XGMI_TIMEOUT_S="2.0")
    cmd = [sys.executable, "-m", "pytorch_distributed_examples_amd.launch.hvdrun", "-np", "2", "--min-np", "1",
           "--verbose", os.path.join(REPO, "horovod_examples", "horovod_mnist_elastic.py"), "--epochs", "2", "--train-size",
           "16384", "--test-size", "1024", "--batches-per-commit", "10"]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=REPO)
    out = res.stdout + res.stderr
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "hvd_elastic_gpu.log"), "w") as f:
        f.write(out)
    assert res.returncode == 0, out[-4000:]
    assert "[fault-injector] rank 1 step 40" in out and "failed (exit 17)" in out, out[-4000:]
    assert "[elastic] reset: world" in out, out[-4000:]
    accs = [ln for ln in res.stdout.splitlines() if ln.startswith("Accuracy:")]
    assert accs and len(set(accs)) == 1, accs  # replicas identical after the recovery
