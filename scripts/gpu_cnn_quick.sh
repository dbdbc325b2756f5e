#!/bin/bash
# Fused-CNN quick check: CNN numerics tests, phase stamps, bench x REPS.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py tests/test_xgmi_gpu.py -q --timeout 120 --timeout-method thread \
  -k "cnn or dropout" > gpurun_out/cnnq_pytest.log 2>&1; rc=$?
grep -E "passed|failed|^E " gpurun_out/cnnq_pytest.log | tail -8
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python scripts/cnn_phase_stamps.py > gpurun_out/cnnq_stamps.log 2>&1; tail -16 gpurun_out/cnnq_stamps.log
MODELS="cnn" CONFIGS="base" REPS=${REPS:-3} STEPS=50 bash scripts/gpu_envsweep.sh && cp gpurun_out/sweep.txt gpurun_out/cnnq_sweep.txt
