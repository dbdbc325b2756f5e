#!/bin/bash
# Round-4 check E: running-statistics diagnostic, then check D (BatchNorm fold tests, benches, kernel table).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 200 python scripts/diag_bn_running.py 2>&1 | grep -v amdgpu.ids | tail -8 || exit 1
bash scripts/runs/archive/gpu_r4d.sh
