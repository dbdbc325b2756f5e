#!/bin/bash
# Round-6 N: BatchNorm fold A/B now that the GEMM cores are spill-free; CNN driver-config repeat (variance).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
bench() {  # label, args...
  local label=$1; shift
  timeout -k 10 200 python bench.py "$@" > gpurun_out/r6n_$label.log 2>&1 || { tail -5 gpurun_out/r6n_$label.log; return 1; }
  echo "$label $(grep '^{' gpurun_out/r6n_$label.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
}
bench cnn_a --steps 20 --warmup 5 || exit 1
bench cnn_b --steps 20 --warmup 5 || exit 1
bench cnn_long --steps 500 --warmup 50 || exit 1
export PDE_BN_FOLD=1
bench resnet50_fold --model resnet50 --steps 30 --warmup 10 || exit 1
bench stage1_fold --model resnet50_stage --stage 1 --batch 8 --steps 40 --warmup 5 || exit 1
bench stage2_fold --model resnet50_stage --stage 2 --batch 8 --steps 40 --warmup 5 || exit 1
unset PDE_BN_FOLD
bench resnet50 --model resnet50 --steps 30 --warmup 10 || exit 1
