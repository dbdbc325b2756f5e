#!/bin/bash
# Round-5 Q: hybrid GEMM core (DMA for 3x3 forward convs / long-K small-M problems, ring elsewhere) A/B on
# ResNet-50 and the m = 8 stages (alternating runs), + numerics under the hybrid core.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
PDE_GEMM_CORE=hybrid timeout -k 10 400 python -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_models_gpu.py > gpurun_out/r5q_pytest.log 2>&1 || { tail -20 gpurun_out/r5q_pytest.log; exit 1; }
tail -1 gpurun_out/r5q_pytest.log
: > gpurun_out/r5q_bench.jsonl
for rep in 1 2; do for core in ring hybrid; do
  for m in "resnet50" "resnet50_stage --stage 1 --batch 8" "resnet50_stage --stage 2 --batch 8" "resnet50_stage --stage 1 --batch 32 --mb-group 4" "resnet50_stage --stage 2 --batch 32 --mb-group 4"; do
    PDE_GEMM_CORE=$core timeout -k 10 200 python bench.py --model $m --steps 30 --warmup 10 > gpurun_out/r5q_one.log 2>&1 || { tail -20 gpurun_out/r5q_one.log; exit 1; }
    tail -1 gpurun_out/r5q_one.log >> gpurun_out/r5q_bench.jsonl
    echo "$core | $m | $(tail -1 gpurun_out/r5q_one.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done; done
