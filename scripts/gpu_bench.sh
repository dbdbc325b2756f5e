#!/bin/bash
# Bench matrix: eager vs hipGraph for each model.  Usage: bash scripts/gpu_bench.sh [models...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
models=${@:-cnn mlp resnet50}
for m in $models; do
  for g in "" "--no-graph"; do
    timeout -k 10 300 python bench.py --model $m --steps 50 --warmup 10 $g 2>&1 | tail -2 || exit 1
  done
done
