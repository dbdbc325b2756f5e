#!/bin/bash
# Round-3 check S: K-slice balancing inside paired backward GEMMs (PDE_GEMM_PAIR_BALANCE): GEMM / conv / ResNet
# tests, then resnet50, stage 1 / 2 (unit 32) and mlp benches on / off.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -q --timeout 300 \
  --timeout-method thread -k "conv or linear or gemm or pair or resnet or mlp" > gpurun_out/r3s_pytest.log 2>&1; rc=$?
grep -E "passed|failed|^E |FAILED" gpurun_out/r3s_pytest.log | tail -12
[ $rc -eq 0 ] || exit 1
MODELS="resnet50 mlp" CONFIGS="base;PDE_GEMM_PAIR_BALANCE=0" REPS=2 bash scripts/gpu_envsweep.sh && cp gpurun_out/sweep.txt gpurun_out/r3s_sweep.txt && \
BENCH_ARGS="--stage 1 --batch 32 --mb-group 4" MODELS="resnet50_stage" CONFIGS="base;PDE_GEMM_PAIR_BALANCE=0" bash scripts/gpu_envsweep.sh && \
  cat gpurun_out/sweep.txt >> gpurun_out/r3s_sweep.txt && \
BENCH_ARGS="--stage 2 --batch 32 --mb-group 4" MODELS="resnet50_stage" CONFIGS="base;PDE_GEMM_PAIR_BALANCE=0" bash scripts/gpu_envsweep.sh && \
  cat gpurun_out/sweep.txt >> gpurun_out/r3s_sweep.txt
