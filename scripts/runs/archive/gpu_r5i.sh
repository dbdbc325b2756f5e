#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 120 python scripts/mlp_mega_phases.py > gpurun_out/r5i_phases.txt 2>&1; rc=$?; cat gpurun_out/r5i_phases.txt; exit $rc
