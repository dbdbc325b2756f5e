#!/bin/bash
# Round-5 ZG (measurement): sub-phase clocks inside the fused MLP backward windows.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 120 python scripts/mlp_mega_phases.py > gpurun_out/r5zg_phases.txt 2>&1 || { tail -20 gpurun_out/r5zg_phases.txt; exit 1; }
tail -8 gpurun_out/r5zg_phases.txt
PDE_MLP_EARLY=0 timeout -k 10 120 python scripts/mlp_mega_phases.py > gpurun_out/r5zg_phases_late.txt 2>&1 || { tail -20 gpurun_out/r5zg_phases_late.txt; exit 1; }
tail -7 gpurun_out/r5zg_phases_late.txt
