#!/bin/bash
# Round-3 check AC: BatchNorm chunks of 5..8 rows per thread kept in registers (PDE_BN_RC8=1)
# BN kernel + ResNet tests with it on, ResNet-50 bench base vs rc8.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
PDE_BN_RC8=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -v --timeout 120 \
  --timeout-method thread -k "batchnorm or resnet" > gpurun_out/r3ac_pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed|^E " gpurun_out/r3ac_pytest.log | tail -20
[ $rc -eq 0 ] || exit 1
MODELS="resnet50" CONFIGS="base;PDE_BN_RC8=1" REPS=3 STEPS=30 bash scripts/gpu_envsweep.sh && cp gpurun_out/sweep.txt gpurun_out/r3ac_sweep.txt
