#!/bin/bash
# Round-3 check K: Adam folded into the MLP's backward GEMM launches (optimiser blocks appended to the pair
# kernels): equivalence test + GEMM/model tests, MLP bench folded vs separate, resnet50 regression, MLP graph trace.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 PYTHONFAULTHANDLER=1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -v --timeout 300 \
  --timeout-method thread -k "folded or mlp or linear or skinny or optim or adam or sgd" > gpurun_out/r3k_pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|^E " gpurun_out/r3k_pytest.log | tail -30
[ $rc -le 1 ] || exit $rc
MODELS="mlp" CONFIGS="base;PDE_MLP_FOLD_OPT=0" STEPS=50 REPS=2 bash scripts/gpu_envsweep.sh && \
  cp gpurun_out/sweep.txt gpurun_out/r3k_sweep_mlp.txt && \
MODELS="resnet50 cnn" CONFIGS="base" bash scripts/gpu_envsweep.sh && cp gpurun_out/sweep.txt gpurun_out/r3k_sweep_other.txt
