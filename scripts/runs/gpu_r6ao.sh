#!/bin/bash
# Round-6 AO: driver-config CNN bench vs hipGraph step-group size (all groups replayed in the warmup).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 PDE_BENCH_PHASES=0 PDE_BENCH_OVERHEADS=0
for rep in 1 2 3; do
  for gs in 1 2 4 5; do
    timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --graph-steps $gs > gpurun_out/r6ao.log 2>&1 || { tail -5 gpurun_out/r6ao.log; exit 1; }
    echo "gs=$gs $(grep '^{' gpurun_out/r6ao.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["steps_per_graph"])')"
  done
done
