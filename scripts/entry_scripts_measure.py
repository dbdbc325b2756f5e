"""Run the reference entry scripts on one GPU with their default (fast) paths and record each epoch's
"images/s (node)" next to the matching ``bench.py --model`` number.

    python scripts/entry_scripts_measure.py OUT.jsonl

Each script runs as a child process (the GPU is initialised there, never here).  The first epoch includes the
hipGraph captures; the steady-state epochs follow it.
"""
import json
import os
import re
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PY = sys.executable

RUNS = [
    ("mnist_ddp_elastic (MLP, default)", [PY, "pytorch_elastic/mnist_ddp_elastic.py", "4", "10",
                                          "--snapshot_path", "/tmp/pde_entry_mlp.pt"], "mlp", 128),
    ("mnist_ddp_elastic --model cnn --batch_size 1024", [PY, "pytorch_elastic/mnist_ddp_elastic.py", "4", "10",
                                                          "--model", "cnn", "--batch_size", "1024",
                                                          "--snapshot_path", "/tmp/pde_entry_cnn.pt"], "cnn", 1024),
    ("mnist_horovod (CNN, SGD, batch 1024)", [PY, "horovod_examples/mnist_horovod.py", "--epochs", "4"], "hvd_cnn", 1024),
]
EPOCH = re.compile(r"Epoch (\d+) \| train ([0-9.]+)s \| ([0-9.]+) images/s \(node\)")


def bench(model):
    out = subprocess.run([PY, "bench.py", "--model", model, "--steps", "200", "--warmup", "20"], cwd=REPO,
                         capture_output=True, text=True, timeout=600)
    for line in out.stdout.splitlines():
        if line.startswith("{"):
            return json.loads(line)
    raise RuntimeError(out.stderr[-2000:])


def main(path):
    with open(path, "w") as f:
        for name, cmd, model, batch in RUNS:
            for a in cmd:
                if a.startswith("/tmp/pde_entry") and os.path.exists(a):
                    os.remove(a)  # a stale snapshot would resume instead of training
            env = dict(os.environ, PYTHONUNBUFFERED="1")
            t = time.time()
            out = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=600, env=env)
            wall = time.time() - t
            if out.returncode != 0:
                raise SystemExit(f"{name} failed rc={out.returncode}:\n{out.stderr[-3000:]}")
            epochs = [dict(epoch=int(m.group(1)), train_s=float(m.group(2)), images_per_s=float(m.group(3)))
                      for m in EPOCH.finditer(out.stdout)]
            b = bench(model)
            steady = [e["images_per_s"] for e in epochs[1:]] or [e["images_per_s"] for e in epochs]
            best = max(steady)
            rec = dict(script=name, cmd=" ".join(cmd[1:]), epochs=epochs, wall_s=round(wall, 2),
                       steady_images_per_s_median=sorted(steady)[len(steady) // 2], steady_images_per_s_best=best,
                       bench_model=model, bench_images_per_s=b["value"], bench_ms_per_step=b["ms_per_step"],
                       ratio_bench_over_script=round(b["value"] / sorted(steady)[len(steady) // 2], 3),
                       printed_tail=out.stdout.splitlines()[-6:])
            f.write(json.dumps(rec) + "\n")
            f.flush()
            print(json.dumps({k: rec[k] for k in ("script", "steady_images_per_s_median", "bench_images_per_s",
                                                 "ratio_bench_over_script")}), flush=True)


if __name__ == "__main__":
    main(sys.argv[1])
