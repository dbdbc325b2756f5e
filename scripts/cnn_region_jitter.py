"""Distribution of the driver-config timed region (bench.py defaults: CNN, K = 20 steps = one 20-step hipGraph
replay) over many regions in ONE process: is the 0.0286 / 0.0328 ms bimodality of single runs per region (host or
device jitter) or per process?  Prints, per region, the region time, the host time of the replay call and the
device time of the replay (events)."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_distributed_examples_amd.bench import harness  # noqa: E402
from pytorch_distributed_examples_amd.parallel import dist as pdist  # noqa: E402

args = harness.parse_args(["--steps", "20", "--warmup", "5"])
ctx = pdist.init_distributed()
work = harness.build_data_parallel(args, ctx, 1024)
harness.run_steps(work, 0, 5)
rows = []
for r in range(int(os.environ.get("REGIONS", "40"))):
    pdist.barrier(ctx)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    harness.run_steps(work, 5, 20)
    e1.record()
    th = time.perf_counter()
    pdist.barrier(ctx)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    rows.append((dt * 1e3 / 20, (th - t0) * 1e3, e0.elapsed_time(e1) / 20))
    if os.environ.get("IDLE_MS"):
        time.sleep(float(os.environ["IDLE_MS"]) / 1e3)
for r in rows:
    print(f"region ms/step {r[0]:.4f}  host call ms {r[1]:.4f}  device ms/step {r[2]:.4f}")
v = [r[0] for r in rows]
print(json.dumps({"regions": len(v), "min": min(v), "median": statistics.median(v), "max": max(v),
                  "device_median": statistics.median(r[2] for r in rows),
                  "host_call_median_ms": statistics.median(r[1] for r in rows)}))
