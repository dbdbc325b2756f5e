#!/bin/bash
# Round-6 O: CNN driver-config region jitter (one process, 40 regions; then with 50 ms idle between regions).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 200 python scripts/cnn_region_jitter.py > gpurun_out/r6o_jitter.log 2>&1 || { tail -5 gpurun_out/r6o_jitter.log; exit 1; }
tail -1 gpurun_out/r6o_jitter.log
IDLE_MS=50 timeout -k 10 200 python scripts/cnn_region_jitter.py > gpurun_out/r6o_jitter_idle.log 2>&1 || { tail -5 gpurun_out/r6o_jitter_idle.log; exit 1; }
tail -1 gpurun_out/r6o_jitter_idle.log
