#!/bin/bash
# Round-3 check D: ResNet numerics with conv->BN slab deferral + downsample GradJoin, parameter-server ring,
# hybrid script, elastic rehearsal; benches (cnn / resnet50 / stages at micro-batch 8, phase timers);
# hipGraph kernel tables of resnet50 and both stages (scripts/gpu_r3c.sh).
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_models_gpu.py tests/test_kernels_gpu.py tests/test_pipeline_gpu.py \
  tests/test_elastic_gpu.py -v --timeout 300 --timeout-method thread \
  -k "resnet or batchnorm or conv or parameter_server or hybrid or elastic" > gpurun_out/r3d_pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r3d_pytest.log | tail -60
[ $rc -le 1 ] || exit $rc
for m in "cnn" "resnet50" "resnet50_stage --stage 1 --batch 8" "resnet50_stage --stage 2 --batch 8"; do
  timeout -k 10 200 python bench.py --model $m --steps 30 --warmup 10 > gpurun_out/r3d_bench_one.log 2>&1 || { tail -20 gpurun_out/r3d_bench_one.log; exit 1; }
  tail -1 gpurun_out/r3d_bench_one.log | tee -a gpurun_out/r3d_bench.jsonl
done
bash scripts/gpu_r3c.sh
