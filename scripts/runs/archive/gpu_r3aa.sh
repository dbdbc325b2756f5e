#!/bin/bash
# Round-3 check AA: BatchNorm tagged-partials hand-off (PDE_BN_TAGGED=1: no ticket, partials stored with an epoch tag and
# polled by every block): BN kernel + ResNet tests with it on, ResNet-50 bench base vs tagged.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
PDE_BN_TAGGED=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -v --timeout 120 \
  --timeout-method thread -k "batchnorm or resnet" > gpurun_out/r3aa_pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed|^E " gpurun_out/r3aa_pytest.log | tail -20
[ $rc -eq 0 ] || exit 1
MODELS="resnet50" CONFIGS="base;PDE_BN_TAGGED=1" REPS=3 STEPS=30 bash scripts/gpu_envsweep.sh && cp gpurun_out/sweep.txt gpurun_out/r3aa_sweep.txt
