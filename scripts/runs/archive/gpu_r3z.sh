#!/bin/bash
# Round-3 check Z: BatchNorm grid sweep with the all-finalize hand-off (blocks per launch / chunk cap).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
MODELS="resnet50" CONFIGS="base;PDE_BN_BLOCKS=512;PDE_BN_BLOCKS=512 PDE_BN_CHUNKS=128;PDE_BN_BLOCKS=128;PDE_BN_CHUNKS=32" \
  REPS=2 STEPS=30 bash scripts/gpu_envsweep.sh && cp gpurun_out/sweep.txt gpurun_out/r3z_sweep.txt
