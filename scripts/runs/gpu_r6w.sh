#!/bin/bash
# Round-6 W: one-launch BatchNorm forward latency by size (graph of 20 calls).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 200 python scripts/bn_latency_bench.py > gpurun_out/r6w_bn_latency.jsonl 2>gpurun_out/r6w_err.log || { tail -5 gpurun_out/r6w_err.log; exit 1; }
cat gpurun_out/r6w_bn_latency.jsonl
PDE_BN_CHUNKS=8 timeout -k 10 200 python scripts/bn_latency_bench.py > gpurun_out/r6w_bn_latency_c8.jsonl 2>>gpurun_out/r6w_err.log || exit 1
echo chunks8; cat gpurun_out/r6w_bn_latency_c8.jsonl
