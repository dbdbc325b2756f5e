#!/bin/bash
# Round-4 check AC: does the fused CNN's end-of-kernel drain wait on P9's narrow slab stores? (timing only)
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for cfg in "PDE_X=0" "PDE_CNN_DIAG_P9ST=1" "PDE_CNN_DIAG_P9ST=1 PDE_CNN_DIAG=1" "PDE_CNN_DIAG=1" "PDE_X=0"; do
  env $cfg timeout -k 10 200 python bench.py --steps 300 --warmup 20 > gpurun_out/r4ac_one.log 2>&1 || { tail -20 gpurun_out/r4ac_one.log; exit 1; }
  tail -1 gpurun_out/r4ac_one.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', d['ms_per_step'], d['value'])"
done
PDE_CNN_DIAG_P9ST=1 timeout -k 10 120 python scripts/cnn_phase_stamps.py 2>&1 | grep -v amdgpu.ids | tail -5
