#!/bin/bash
# Round-4 check Z: what the CNN reduction launch spends on the SGD update / fragment refresh (PDE_CNN_DIAG=16).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for d in 0 16 20 24 1 0; do
  PDE_CNN_DIAG=$d timeout -k 10 200 python bench.py --steps 300 --warmup 20 > gpurun_out/r4z_one.log 2>&1 || { tail -20 gpurun_out/r4z_one.log; exit 1; }
  tail -1 gpurun_out/r4z_one.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('diag=$d', d['ms_per_step'], d['value'])"
done
