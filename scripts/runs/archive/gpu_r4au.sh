#!/bin/bash
# Round-4 check AU: conv2-dgrad B fragments from the vector-memory path (PDE_CNN_BREG=1) now that the phase is
# LDS-bound -- A/B bench + stamps, default first.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for breg in 0 1 0 1; do
  PDE_CNN_BREG=$breg timeout -k 10 200 python bench.py --steps 300 --warmup 20 > gpurun_out/r4au_one.log 2>&1 || { tail -20 gpurun_out/r4au_one.log; exit 1; }
  echo "BREG=$breg $(tail -1 gpurun_out/r4au_one.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'])")"
done
PDE_CNN_BREG=1 timeout -k 10 120 python scripts/cnn_phase_stamps.py 2>&1 | grep -v amdgpu.ids | grep -E "P7|P9|total"
