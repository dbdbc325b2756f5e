"""bench.py output contract (one JSON line, required fields), exercised on CPU: 1 rank and 2 ranks
under torchrun (gloo)."""
import json
import re
import os

from dist_utils import REPO, free_port, run_cmd

FIELDS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
          "scaling", "vs_baseline", "dtype", "data", "config"}



def _rec(line):
    """The JSON record at the start of a line (another rank's log text may follow it on the same line)."""
    return json.JSONDecoder().raw_decode(line)[0]

def _parse(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    rec = json.loads(lines[0])
    assert FIELDS <= set(rec), rec
    assert {"model", "global_batch", "seq_len", "parallelism"} <= set(rec["config"])
    return rec


def test_bench_cpu_single():
    rc, out = run_cmd(["python", os.path.join(REPO, "bench.py"), "--device", "cpu", "--steps", "2", "--warmup", "1",
                       "--batch", "32"], timeout=300)
    assert rc == 0, out
    rec = _parse(out)
    assert rec["n_gpus"] == 1 and rec["steps"] == 2 and rec["warmup"] == 1 and rec["value"] > 0
    assert rec["config"]["global_batch"] == 32 and rec["config"]["parallelism"] == "dp1"


def test_bench_cpu_torchrun_world2():
    rc, out = run_cmd(["python", "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                       "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(REPO, "bench.py"),
                       "--gpus", "2", "--device", "cpu", "--steps", "2", "--warmup", "1",
                       "--model", "mlp"], timeout=300)
    assert rc == 0, out
    rec = _parse(out)
    # the reference's MLP DDP at world 2 (CPU) is the same workload: vs_baseline is reported
    assert rec["n_gpus"] == 2 and rec["config"]["global_batch"] == 256 and rec["vs_baseline"] is not None


def test_bench_launches_n_ranks_itself():
    """``bench.py --gpus 2`` without torchrun launches 2 ranks (the driver's N-GPU contract)."""
    rc, out = run_cmd(["python", os.path.join(REPO, "bench.py"), "--gpus", "2", "--device", "cpu", "--steps", "2",
                       "--warmup", "1", "--batch", "16", "--model", "mlp"], timeout=300)
    assert rc == 0, out
    rec = _parse(out)
    assert rec["n_gpus"] == 2 and rec["config"]["rccl_nranks"] == 2 and rec["config"]["parallelism"] == "dp2"


def test_bench_world_mismatch_fails_fast():
    rc, out = run_cmd(["python", "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                       "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(REPO, "bench.py"),
                       "--gpus", "4", "--device", "cpu", "--steps", "1", "--warmup", "0"], timeout=300)
    assert rc != 0 and "--gpus 4 but the job has 2 ranks" in out, out


def test_bench_resnet_pipeline_world2():
    """BASELINE config 3 plumbing: 2-stage ResNet-50 pipeline, one rank per stage (tiny images on CPU)."""
    rc, out = run_cmd(["python", os.path.join(REPO, "bench.py"), "--gpus", "2", "--device", "cpu", "--steps", "2",
                       "--warmup", "1", "--model", "resnet50_pp", "--batch", "4", "--split-size", "2",
                       "--image", "32"], timeout=300)
    assert rc == 0, out
    rec = _parse(out)
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "pp2xdp1" and rec["config"]["microbatches"] == 2
    assert rec["config"]["global_batch"] == 4 and rec["value"] > 0


def test_bench_secondary_pipeline_measurement():
    """At N >= 2 the headline run also measures BASELINE config 3/4 (resnet50_pp) in child processes and
    reports it under config.secondary (forced on CPU here, tiny images)."""
    env = {"PDE_BENCH_SECONDARY": "force",
           "PDE_BENCH_SECONDARY_ARGS": "--device cpu --batch 4 --split-size 2 --image 32 --steps 1 --warmup 1"}
    rc, out = run_cmd(["python", os.path.join(REPO, "bench.py"), "--gpus", "2", "--device", "cpu", "--steps", "2",
                       "--warmup", "1", "--batch", "16"], timeout=300, env=env)
    assert rc == 0, out
    rec = _parse(out)
    sec = rec["config"]["secondary"]
    assert "error" not in sec, sec
    assert sec["parallelism"] == "pp2xdp1" and sec["value"] > 0 and sec["global_batch"] == 4


def test_bench_elastic_scale_up_cpu():
    """BASELINE config 2 contract: ``bench.py --model elastic_cnn --gpus 2 --scale-to 4`` starts 2 workers
    under the elastic driver, scales to 4 mid-run WITHOUT restarting the first two (in-process re-wire),
    prints one JSON line per round and the final contract line with every round's img/s and re-wire latency."""
    rc, out = run_cmd(["python", os.path.join(REPO, "bench.py"), "--model", "elastic_cnn", "--gpus", "2",
                       "--scale-to", "4", "--device", "cpu", "--batch", "32", "--steps", "4", "--warmup", "2",
                       "--graph-steps", "2"], timeout=600)
    assert rc == 0, out
    rounds = [_rec(ln) for ln in out.splitlines() if ln.startswith('{"event": "round"')]
    final = [_rec(ln) for ln in out.splitlines() if ln.startswith('{"metric"')]
    assert len(final) == 1 and FIELDS <= set(final[0]), out
    rec = final[0]
    assert [r["world"] for r in rounds] == [2, 4] and rec["n_gpus"] == 4, out
    assert rounds[0]["rewire_s"] is None and rounds[1]["rewire_s"] > 0
    assert all(r["images_per_s"] > 0 for r in rec["config"]["rounds"])
    # the first round's workers survived the membership change (same pids in both rounds)
    pids = {}
    for ln in out.splitlines():
        if ln.startswith("[rewire] round ") and "(pid " in ln:
            rnd = int(ln.split()[2].rstrip(":"))
            pids.setdefault(rnd, set()).add(int(re.match(r"\d+", ln.split("(pid ")[1]).group(0)))
    assert pids[0] <= pids[1] and len(pids[1]) == 4, pids


def test_bench_elastic_survives_killed_worker_cpu():
    """BASELINE config 2 failure rehearsal (horovod/horovod_mnist_elastic.py:55,104-106 semantics): rank 1 exits
    mid-run (``--fault-at``); the survivor turns the failed collective into PeerFailure, restores its commit,
    re-joins at world 1 in the SAME process and times the new round, reporting the re-wire latency and its
    parts (rendezvous / control group / broadcast / map / capture)."""
    rc, out = run_cmd(["python", os.path.join(REPO, "bench.py"), "--model", "elastic_cnn", "--gpus", "2",
                       "--scale-to", "1", "--fault-at", "20", "--device", "cpu", "--batch", "32", "--steps", "4",
                       "--warmup", "2", "--graph-steps", "2"], timeout=600)
    assert rc == 0, out[-4000:]
    rounds = [_rec(ln) for ln in out.splitlines() if ln.startswith('{"event": "round"')]
    final = [_rec(ln) for ln in out.splitlines() if ln.startswith('{"metric"')]
    assert "[fault-injector] rank 1 step 20" in out and "peer failure" in out, out[-4000:]
    assert [r["world"] for r in rounds] == [2, 1] and len(final) == 1, out[-4000:]
    assert rounds[1]["rewire_s"] > 0 and set(rounds[1]["rewire_parts"]) == {
        "rendezvous_s", "control_s", "broadcast_s", "map_s", "capture_s", "detect_s"}, rounds[1]
    # detection: the fault -> PeerFailure latency (driver's failure report -> abort word / commit point)
    assert 0 < rounds[1]["rewire_parts"]["detect_s"] < 10.0, rounds[1]
    assert "worker killed" in final[0]["config"]["parallelism"]
    pids = {}
    for ln in out.splitlines():
        if ln.startswith("[rewire] round ") and "(pid " in ln:
            rnd = int(ln.split()[2].rstrip(":"))
            pids.setdefault(rnd, set()).add(int(re.match(r"\d+", ln.split("(pid ")[1]).group(0)))
    assert pids[1] < pids[0], pids  # the survivor kept its process


def test_auto_graph_group_is_replayed_by_the_warmup():
    """The auto hipGraph step group is the largest divisor of --steps up to --warmup (when that keeps >= 4 steps per
    graph), so the timed region never holds a graph's first replay; otherwise the largest divisor up to 50."""
    from pytorch_distributed_examples_amd.bench.harness import parse_args

    cases = {(20, 5): 5, (100, 20): 20, (300, 30): 30, (500, 50): 50, (7, 5): 7, (20, 2): 20, (20, 0): 20, (64, 12): 8}
    for (steps, warmup), want in cases.items():
        a = parse_args(["--steps", str(steps), "--warmup", str(warmup)])
        assert a.graph_steps == want, (steps, warmup, a.graph_steps)
        assert steps % a.graph_steps == 0
    assert parse_args(["--steps", "20", "--warmup", "5", "--graph-steps", "10"]).graph_steps == 10
