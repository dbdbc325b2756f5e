#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 120 python scripts/mlp_mega_diag.py > gpurun_out/r5n_diag.txt 2>&1 || { tail -20 gpurun_out/r5n_diag.txt; exit 1; }
PDE_MLP_PRELOAD=0 timeout -k 10 120 python scripts/mlp_mega_diag.py > gpurun_out/r5n_diag_nopre.txt 2>&1 || { tail -20 gpurun_out/r5n_diag_nopre.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r5n_diag.txt; echo ---- no preload; grep -v amdgpu.ids gpurun_out/r5n_diag_nopre.txt
