#!/bin/bash
# Round-5 ZM: HBM bytes of the one-launch MLP step (FETCH_SIZE / WRITE_SIZE, one counter pass each).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p "$R/gpurun_out"
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/r5zm_fetch" -o f -- python3 "$R/bench.py" --model mlp --steps 20 --warmup 5 --no-graph \
  > "$R/gpurun_out/r5zm_fetch.log" 2>&1 || { tail -20 "$R/gpurun_out/r5zm_fetch.log"; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/r5zm_write" -o w -- python3 "$R/bench.py" --model mlp --steps 20 --warmup 5 --no-graph \
  > "$R/gpurun_out/r5zm_write.log" 2>&1 || { tail -20 "$R/gpurun_out/r5zm_write.log"; exit 1; }
cd "$R"
python3 - <<'PY'
import csv, glob, statistics
for tag, d in (("FETCH_SIZE", "gpurun_out/r5zm_fetch"), ("WRITE_SIZE", "gpurun_out/r5zm_write")):
    fs = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    vals = []
    for f in fs:
        for r in csv.DictReader(open(f)):
            if "k_mlp_train" in r.get("Kernel_Name", "") and r.get("Counter_Name") == tag:
                vals.append(float(r["Counter_Value"]))
    print(tag, "dispatches", len(vals), "median KB", statistics.median(vals) if vals else None)
PY
