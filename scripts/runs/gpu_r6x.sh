#!/bin/bash
# Round-6 X: in-launch split-K combine (now spill-free) vs the separate slab-reduce launch: stage / ResNet A/B.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
bench() {  # label, args...
  local label=$1; shift
  timeout -k 10 200 python bench.py "$@" > gpurun_out/r6x_$label.log 2>&1 || { tail -5 gpurun_out/r6x_$label.log; return 1; }
  echo "$label $(grep '^{' gpurun_out/r6x_$label.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
}
for rep in 1 2; do
  bench stage2_off$rep --model resnet50_stage --stage 2 --batch 8 --steps 40 --warmup 5 || exit 1
  PDE_GEMM_INKERNEL_SPLITK=1 bench stage2_on$rep --model resnet50_stage --stage 2 --batch 8 --steps 40 --warmup 5 || exit 1
done
bench stage1_off --model resnet50_stage --stage 1 --batch 8 --steps 40 --warmup 5 || exit 1
PDE_GEMM_INKERNEL_SPLITK=1 bench stage1_on --model resnet50_stage --stage 1 --batch 8 --steps 40 --warmup 5 || exit 1
bench resnet50_off --model resnet50 --steps 30 --warmup 10 || exit 1
PDE_GEMM_INKERNEL_SPLITK=1 bench resnet50_on --model resnet50 --steps 30 --warmup 10 || exit 1
PDE_GEMM_INKERNEL_SPLITK=1 bench mlp_on --model mlp --steps 100 --warmup 20 || exit 1
