#!/bin/bash
# Round-3 check AB: fused CNN tail with the lite grid barrier (write-through slab stores, coherent loads, no
# L2 write-back / invalidate): CNN tests, bench base (two launches) vs PDE_CNN_FUSED_TAIL=1.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py tests/test_xgmi_gpu.py -v --timeout 120 --timeout-method thread \
  -k "cnn or dropout" > gpurun_out/r3ab_pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed|^E " gpurun_out/r3ab_pytest.log | tail -16
[ $rc -eq 0 ] || exit 1
MODELS="cnn" CONFIGS="base;PDE_CNN_FUSED_TAIL=1" REPS=3 STEPS=100 bash scripts/gpu_envsweep.sh && cp gpurun_out/sweep.txt gpurun_out/r3ab_sweep.txt
