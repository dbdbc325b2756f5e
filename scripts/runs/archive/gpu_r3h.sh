#!/bin/bash
# Round-3 check H: grouped-BN block test + pipeline rehearsals (reference with the same units), GEMM / MLP tests
# after the narrow-problem pairing change, then BatchNorm-grid and optimizer env sweeps (resnet50 / mlp).
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 PYTHONFAULTHANDLER=1
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_pipeline_gpu.py \
  -v --timeout 300 --timeout-method thread -k "grouped or rehearsal or linear or gemm or mlp or pair" > gpurun_out/r3h_pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r3h_pytest.log | tail -40
[ $rc -le 1 ] || exit $rc
MODELS="resnet50" CONFIGS="base;PDE_BN_CHUNKS=256;PDE_BN_BLOCKS=512;PDE_BN_CHUNKS=256 PDE_BN_BLOCKS=512" bash scripts/gpu_envsweep.sh && \
  cp gpurun_out/sweep.txt gpurun_out/r3h_sweep_resnet.txt && \
MODELS="mlp" CONFIGS="base;PDE_OPTIM_NT=0;PDE_OPTIM_BLOCKS=2048;PDE_OPTIM_BLOCKS=512;PDE_GEMM_PAIR=0" STEPS=50 bash scripts/gpu_envsweep.sh && \
  cp gpurun_out/sweep.txt gpurun_out/r3h_sweep_mlp.txt
