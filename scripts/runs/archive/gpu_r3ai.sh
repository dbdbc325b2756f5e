#!/bin/bash
# Round-3 check AI: MSE forward with 8 loads in flight per thread, CE rows in registers: loss tests, ResNet tests, bench.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -v --timeout 120 \
  --timeout-method thread -k "mse or loss or resnet or fused_mlp or cross" > gpurun_out/r3ai_pytest.log 2>&1; rc=$?
grep -E "FAILED|passed|failed|^E " gpurun_out/r3ai_pytest.log | tail -12
[ $rc -eq 0 ] || exit 1
MODELS="resnet50 mlp" CONFIGS="base" REPS=3 STEPS=30 bash scripts/gpu_envsweep.sh && cp gpurun_out/sweep.txt gpurun_out/r3ai_sweep.txt
