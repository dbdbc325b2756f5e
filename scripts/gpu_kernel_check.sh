#!/bin/bash
# Focused GPU check for kernel work: kernel + model tests, the MLP and ResNet-50 benches, ResNet-50 rocprof.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_models_gpu.py > gpurun_out/pytest_k.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_k.log | tail -30; [ $rc -eq 0 ] || exit $rc
for m in ${BENCH_MODELS:-mlp resnet50}; do
  timeout -k 10 300 python bench.py --model $m --steps 30 --warmup 10 > gpurun_out/bench_$m.log 2>&1 || { tail -20 gpurun_out/bench_$m.log; exit 1; }
  tail -1 gpurun_out/bench_$m.log
done
bash scripts/gpu_profile.sh ${PROFILE_MODELS:-resnet50}
