#!/bin/bash
# Round-4 check N: MLP step vs the fused optimiser's grid size / load-store flavour / folding into the GEMMs.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
: > gpurun_out/r4n_bench.txt
run() {
  local label=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 200 python bench.py "$@" > gpurun_out/r4n_one.log 2>&1 || { tail -20 gpurun_out/r4n_one.log; return 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4n_one.log').read().strip().splitlines()[-1]); print('$label', d['config']['model'], d['ms_per_step'], d['value'])" | tee -a gpurun_out/r4n_bench.txt
}
for cfg in "PDE_OPTIM_BLOCKS=768" "PDE_OPTIM_BLOCKS=256" "PDE_OPTIM_BLOCKS=512" "PDE_OPTIM_BLOCKS=1224" "PDE_OPTIM_NT=0" "PDE_OPTIM_NT=0 PDE_OPTIM_BLOCKS=1224" "PDE_MLP_FOLD_OPT=1" "PDE_OPTIM_BLOCKS=768"; do
  run "$cfg" $cfg -- --model mlp --steps 100 --warmup 20 || exit 1
done
