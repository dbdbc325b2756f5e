#!/bin/bash
# GEMM tile-policy sweep: kernel/model GPU tests, then the ResNet-50 and MLP benches under PDE_GEMM_*
# overrides (each config is a list of VAR=value assignments; "-" = built-in defaults).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_models_gpu.py > gpurun_out/pytest_k.log 2>&1 || { tail -30 gpurun_out/pytest_k.log; exit 1; }
tail -1 gpurun_out/pytest_k.log
: > gpurun_out/gemm_sweep.txt
for cfg in "${@:--}"; do
  envs=(); [ "$cfg" = "-" ] || envs=($cfg)
  for m in resnet50 mlp; do
    env "${envs[@]}" timeout -k 10 180 python bench.py --model $m --steps 30 --warmup 10 > gpurun_out/sweep_one.log 2>&1 || { tail -20 gpurun_out/sweep_one.log; exit 1; }
    ms=$(tail -1 gpurun_out/sweep_one.log | python -c "import sys,json; print(json.loads(sys.stdin.read())['ms_per_step'])") || exit 1
    echo "cfg=[$cfg] model=$m ms_per_step=$ms" | tee -a gpurun_out/gemm_sweep.txt
  done
done
