#!/bin/bash
# Round-4 check L: write-through stores in the GEMM epilogues (PDE_GEMM_WT=1) and the fused optimiser
# (PDE_OPTIM_NT=2) -- kernel tests with both on, then MLP / ResNet-50 / CNN benches A/B.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
PDE_GEMM_WT=1 PDE_OPTIM_NT=2 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r4l_pytest.log 2>&1 || { tail -30 gpurun_out/r4l_pytest.log; exit 1; }
tail -1 gpurun_out/r4l_pytest.log
: > gpurun_out/r4l_bench.txt
run() {  # label, env..., -- bench args
  local label=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 200 python bench.py "$@" > gpurun_out/r4l_one.log 2>&1 || { tail -20 gpurun_out/r4l_one.log; return 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4l_one.log').read().strip().splitlines()[-1]); print('$label', d['config']['model'], d['ms_per_step'], d['value'])" | tee -a gpurun_out/r4l_bench.txt
}
for rep in 1 2; do
  for cfg in "PDE_GEMM_WT=0 PDE_OPTIM_NT=1" "PDE_GEMM_WT=1 PDE_OPTIM_NT=1" "PDE_GEMM_WT=0 PDE_OPTIM_NT=2" "PDE_GEMM_WT=1 PDE_OPTIM_NT=2"; do
    run "$cfg" $cfg -- --model mlp --steps 100 --warmup 20 || exit 1
    run "$cfg" $cfg -- --model resnet50 --steps 30 --warmup 10 || exit 1
  done
done
run "cnn default" PDE_X=0 -- --steps 200 --warmup 20 || exit 1
