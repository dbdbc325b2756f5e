#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && mkdir -p gpurun_out
PDE_GEMM_LOG=1 timeout -k 10 120 python -u scripts/dbg/dbg_defer.py > gpurun_out/r6ab.log 2>&1; echo rc=$?
grep -v "^\[W\|amdgpu.ids" gpurun_out/r6ab.log | head -60
