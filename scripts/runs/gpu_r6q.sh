#!/bin/bash
# Round-6 Q: low-K GEMM microbench (plain 8-byte stores) vs the tile core; grid-cap sweep.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 120 python scripts/gemm_lowk_bench.py > gpurun_out/r6q_lowk.jsonl 2>gpurun_out/r6q_err.log || { tail -5 gpurun_out/r6q_err.log; exit 1; }
PDE_GEMM_LOWK=0 timeout -k 10 120 python scripts/gemm_lowk_bench.py >> gpurun_out/r6q_lowk.jsonl 2>>gpurun_out/r6q_err.log || exit 1
for b in 256 1024 2048; do PDE_GEMM_LOWK_BLOCKS=$b timeout -k 10 120 python scripts/gemm_lowk_bench.py >> gpurun_out/r6q_lowk.jsonl 2>>gpurun_out/r6q_err.log || exit 1; done
cat gpurun_out/r6q_lowk.jsonl
