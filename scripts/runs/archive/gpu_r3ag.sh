#!/bin/bash
# Round-3 check AG: BatchNorm block target with the 128-chunk tagged hand-off (ResNet-50 + the m8 stage 2).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
MODELS="resnet50" CONFIGS="base;PDE_BN_BLOCKS=384;PDE_BN_BLOCKS=512" REPS=2 STEPS=30 bash scripts/gpu_envsweep.sh && cp gpurun_out/sweep.txt gpurun_out/r3ag_sweep.txt
MODELS="resnet50_stage" BENCH_ARGS="--stage 2 --batch 8" CONFIGS="base;PDE_BN_BLOCKS=512;PDE_BN_CHUNKS=64" REPS=2 STEPS=30 bash scripts/gpu_envsweep.sh && cat gpurun_out/sweep.txt >> gpurun_out/r3ag_sweep.txt
