#!/bin/bash
# Round-5 ZF (measurement): are the fused MLP windows bound by their stores?  PDE_MLP_NOGW=1 drops the p.grad stores.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
PDE_MLP_NOGW=1 timeout -k 10 120 python scripts/mlp_mega_phases.py > gpurun_out/r5zf_phases_nogw.txt 2>&1 || { tail -20 gpurun_out/r5zf_phases_nogw.txt; exit 1; }
grep -E "^B|sum" gpurun_out/r5zf_phases_nogw.txt
for rep in 1 2; do for g in 1 0; do
  PDE_MLP_NOGW=$g timeout -k 10 200 python bench.py --model mlp --steps 200 --warmup 20 > gpurun_out/r5zf_one.log 2>&1 || { tail -20 gpurun_out/r5zf_one.log; exit 1; }
  echo "nogw=$g $(tail -1 gpurun_out/r5zf_one.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done; done
