#!/bin/bash
# Round-4 check Y: optimiser loads / stores plain by default -- ResNet-50 / stage / MLP / CNN A/B vs non-temporal.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
: > gpurun_out/r4y_bench.txt
run() {
  local label=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 200 python bench.py "$@" > gpurun_out/r4y_one.log 2>&1 || { tail -20 gpurun_out/r4y_one.log; return 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4y_one.log').read().strip().splitlines()[-1]); print('$label', d['config']['model'], d['ms_per_step'], d['value'], d['config'].get('phases', {}).get('rank0_ms'))" | tee -a gpurun_out/r4y_bench.txt
}
for rep in 1 2; do for cfg in "PDE_OPTIM_NT=0" "PDE_OPTIM_NT=1"; do
  run "$cfg" $cfg -- --model resnet50 --steps 30 --warmup 10 || exit 1
  run "$cfg" $cfg -- --model mlp --steps 100 --warmup 20 || exit 1
done; done
run "default" PDE_X=0 -- --model resnet50_stage --stage 1 --batch 8 --steps 30 --warmup 10 || exit 1
run "default" PDE_X=0 -- --model resnet50_stage --stage 2 --batch 8 --steps 30 --warmup 10 || exit 1
run "default" PDE_X=0 -- --steps 200 --warmup 20 || exit 1
