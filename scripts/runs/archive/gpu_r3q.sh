#!/bin/bash
# Round-3 check Q: KxK conv weight layout kernel with all tile loads in flight: layout / optimizer tests,
# resnet50 + stage-2 (unit 32) benches, resnet50 graph kernel table.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -q --timeout 300 \
  --timeout-method thread -k "conv or optim or resnet or layout" > gpurun_out/r3q_pytest.log 2>&1; rc=$?
grep -E "passed|failed|^E |FAILED" gpurun_out/r3q_pytest.log | tail -12
[ $rc -eq 0 ] || exit 1
MODELS="resnet50" CONFIGS="base" REPS=2 bash scripts/gpu_envsweep.sh && cp gpurun_out/sweep.txt gpurun_out/r3q_sweep_resnet.txt && \
BENCH_ARGS="--stage 2 --batch 32 --mb-group 4" MODELS="resnet50_stage" CONFIGS="base" bash scripts/gpu_envsweep.sh && \
  cp gpurun_out/sweep.txt gpurun_out/r3q_sweep_stage2.txt
