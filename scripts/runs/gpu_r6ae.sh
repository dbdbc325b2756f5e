#!/bin/bash
# Round-6 AE: driver-config CNN bench, 6 processes each: default 20-step graph (first replayed inside the timed
# region) vs a 5-step graph (replayed once in the warmup).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 PDE_BENCH_PHASES=0 PDE_BENCH_OVERHEADS=0
for rep in 1 2 3 4 5 6; do
  for gs in 0; do
    timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --graph-steps $gs > gpurun_out/r6ae.log 2>&1 || { tail -5 gpurun_out/r6ae.log; exit 1; }
    echo "gs=$gs $(grep '^{' gpurun_out/r6ae.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["steps_per_graph"])')"
  done
done
