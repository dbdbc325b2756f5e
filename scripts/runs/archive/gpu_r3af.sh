#!/bin/bash
# Round-3 check AF: tagged BatchNorm with up to 128 row chunks (PDE_BN_CHUNKS=128: C <= 128 layers get more blocks)
# BN kernel + ResNet tests with it on, ResNet-50 bench base vs chunks 128 / 96.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
PDE_BN_CHUNKS=128 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -v --timeout 120 \
  --timeout-method thread -k "batchnorm or resnet" > gpurun_out/r3af_pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed|^E " gpurun_out/r3af_pytest.log | tail -20
[ $rc -eq 0 ] || exit 1
MODELS="resnet50" CONFIGS="base;PDE_BN_CHUNKS=128;PDE_BN_CHUNKS=96" REPS=2 STEPS=30 bash scripts/gpu_envsweep.sh && cp gpurun_out/sweep.txt gpurun_out/r3af_sweep.txt
