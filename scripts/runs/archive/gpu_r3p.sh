#!/bin/bash
# Round-3 check P: register-cached one-launch BatchNorm forward: BN / ResNet tests, then resnet50 + stage benches
# with the variant on and off (PDE_BN_FWD_RC).
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_pipeline_gpu.py -q \
  --timeout 300 --timeout-method thread -k "batchnorm or resnet or rehearsal" > gpurun_out/r3p_pytest.log 2>&1; rc=$?
grep -E "passed|failed|^E |FAILED" gpurun_out/r3p_pytest.log | tail -12
[ $rc -eq 0 ] || exit 1
MODELS="resnet50" CONFIGS="base;PDE_BN_FWD_RC=0" REPS=2 bash scripts/gpu_envsweep.sh && cp gpurun_out/sweep.txt gpurun_out/r3p_sweep_resnet.txt && \
BENCH_ARGS="--stage 2 --batch 32 --mb-group 4" MODELS="resnet50_stage" CONFIGS="base;PDE_BN_FWD_RC=0" bash scripts/gpu_envsweep.sh && \
  cp gpurun_out/sweep.txt gpurun_out/r3p_sweep_stage2.txt
