#!/bin/bash
# Round-5 T: first weight-gradient write after zero_grad stores instead of read-modify-writing -- numerics + benches
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_streams_gpu.py tests/test_comm_gpu.py > gpurun_out/r5t_pytest.log 2>&1 || { tail -30 gpurun_out/r5t_pytest.log; exit 1; }
tail -1 gpurun_out/r5t_pytest.log
: > gpurun_out/r5t_bench.jsonl
for m in "resnet50" "resnet50_stage --stage 1 --batch 8" "resnet50_stage --stage 2 --batch 8" "resnet50_stage --stage 1 --batch 32 --mb-group 4" "resnet50_stage --stage 2 --batch 32 --mb-group 4" "resnet50"; do
  timeout -k 10 200 python bench.py --model $m --steps 30 --warmup 10 > gpurun_out/r5t_one.log 2>&1 || { tail -20 gpurun_out/r5t_one.log; exit 1; }
  tail -1 gpurun_out/r5t_one.log >> gpurun_out/r5t_bench.jsonl
  echo "$m | $(tail -1 gpurun_out/r5t_one.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done
bash scripts/runs/archive/gpu_r5s.sh
