#!/bin/bash
# Round-3 check U: BatchNorm finalize tail reading up to 256 chunks in one round trip; chunk-cap sweep.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -q --timeout 300 \
  --timeout-method thread -k "batchnorm or resnet_blocks" > gpurun_out/r3u_pytest.log 2>&1; rc=$?
grep -E "passed|failed|^E |FAILED" gpurun_out/r3u_pytest.log | tail -12
[ $rc -eq 0 ] || exit 1
MODELS="resnet50" CONFIGS="base;PDE_BN_CHUNKS=128;PDE_BN_CHUNKS=256" REPS=2 bash scripts/gpu_envsweep.sh && cp gpurun_out/sweep.txt gpurun_out/r3u_sweep.txt && \
BENCH_ARGS="--stage 1 --batch 32 --mb-group 4" MODELS="resnet50_stage" CONFIGS="base;PDE_BN_CHUNKS=256" bash scripts/gpu_envsweep.sh && \
  cat gpurun_out/sweep.txt >> gpurun_out/r3u_sweep.txt
