#!/bin/bash
# Round-3 check A: xGMI epoch fix, CNN dropout masks, P2P ring / pipeline / parameter-server rehearsals,
# one-launch BatchNorm (kernel + ResNet model tests), then the CNN and ResNet-50 benches.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_xgmi_gpu.py \
  tests/test_pipeline_gpu.py -v --timeout 300 --timeout-method thread \
  -k "batchnorm or resnet or xgmi or dropout or fused_cnn or ring or pipeline or parameter_server or hybrid" > gpurun_out/r3a_pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r3a_pytest.log | tail -40
[ $rc -le 1 ] || exit $rc
for m in cnn resnet50; do
  timeout -k 10 200 python bench.py --model $m --steps 30 --warmup 10 > gpurun_out/r3a_bench_$m.log 2>&1 || { tail -20 gpurun_out/r3a_bench_$m.log; exit 1; }
  tail -1 gpurun_out/r3a_bench_$m.log
done
