"""bench.py output contract (one JSON line, required fields), exercised on CPU: 1 rank and 2 ranks
under torchrun (gloo)."""
import json
import os

from dist_utils import REPO, free_port, run_cmd

FIELDS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
          "scaling", "vs_baseline", "dtype", "data", "config"}


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
                       "--gpus", "2", "--device", "cpu", "--steps", "2", "--warmup", "1", "--batch", "32",
                       "--model", "mlp"], timeout=300)
    assert rc == 0, out
    rec = _parse(out)
    assert rec["n_gpus"] == 2 and rec["config"]["global_batch"] == 64 and rec["vs_baseline"] is not None
