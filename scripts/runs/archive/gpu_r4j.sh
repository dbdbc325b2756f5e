#!/bin/bash
# Round-4 check J: where the fused CNN step's time goes between its two launches (PDE_CNN_DIAG: 1 train only,
# 2 reduce only, 4 reduce slab roles only, 8 reduce fc1 roles only; timing only, results invalid).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
: > gpurun_out/r4j_bench.txt
for d in 0 1 2 4 8 0; do
  PDE_CNN_DIAG=$d timeout -k 10 200 python bench.py --steps 200 --warmup 20 > gpurun_out/r4j_one.log 2>&1 || { tail -20 gpurun_out/r4j_one.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4j_one.log').read().strip().splitlines()[-1]); print('diag=$d', d['ms_per_step'], d['value'])" | tee -a gpurun_out/r4j_bench.txt
done
timeout -k 10 120 python scripts/cnn_phase_stamps.py > gpurun_out/r4j_stamps.txt 2>&1 || { tail -20 gpurun_out/r4j_stamps.txt; exit 1; }
cat gpurun_out/r4j_stamps.txt
