#!/bin/bash
# Round-3 check G: grouped BatchNorm (kernel test, pipeline rehearsals with 1/2/4 micro-batches per unit),
# BatchNorm / ResNet model tests, then stage benches of a batch-32 unit = 4 x m8 / 8 x m4 micro-batches.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 PYTHONFAULTHANDLER=1
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_pipeline_gpu.py \
  -v --timeout 300 --timeout-method thread -k "batchnorm or resnet or pipeline" > gpurun_out/r3g_pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r3g_pytest.log | tail -40
[ $rc -le 1 ] || exit $rc
: > gpurun_out/r3g_bench.jsonl
for m in "resnet50_stage --stage 1 --batch 32 --mb-group 4" "resnet50_stage --stage 2 --batch 32 --mb-group 4" \
         "resnet50_stage --stage 1 --batch 32 --mb-group 8" "resnet50_stage --stage 2 --batch 32 --mb-group 8" \
         "resnet50"; do
  timeout -k 10 200 python bench.py --model $m --steps 30 --warmup 10 > gpurun_out/r3g_one.log 2>&1 || { tail -30 gpurun_out/r3g_one.log; exit 1; }
  tail -1 gpurun_out/r3g_one.log >> gpurun_out/r3g_bench.jsonl
  tail -1 gpurun_out/r3g_one.log | cut -c1-200
done
