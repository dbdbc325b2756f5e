#!/bin/bash
# Round-5 Y: split_min_kt 8 by default -- GEMM / model numerics, the pipeline-unit table and the model benches.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_streams_gpu.py > gpurun_out/r5y_pytest.log 2>&1 || { tail -30 gpurun_out/r5y_pytest.log; exit 1; }
tail -1 gpurun_out/r5y_pytest.log
: > gpurun_out/r5y_stages.jsonl
for g in 1 2 4; do for s in 1 2; do
  timeout -k 10 200 python bench.py --model resnet50_stage --stage $s --batch $((8 * g)) --mb-group $g --steps 30 --warmup 10 \
    > gpurun_out/r5y_one.log 2>&1 || { tail -20 gpurun_out/r5y_one.log; exit 1; }
  tail -1 gpurun_out/r5y_one.log >> gpurun_out/r5y_stages.jsonl
done; done
timeout -k 10 200 python bench.py --model resnet50 --steps 30 --warmup 10 > gpurun_out/r5y_one.log 2>&1 || { tail -20 gpurun_out/r5y_one.log; exit 1; }
tail -1 gpurun_out/r5y_one.log > gpurun_out/r5y_resnet50.jsonl
python3 scripts/pipeline_units.py gpurun_out/r5y_stages.jsonl --one-gpu gpurun_out/r5y_resnet50.jsonl --json gpurun_out/r5y_pipeline_units.json \
  > gpurun_out/r5y_pipeline_units.md && cat gpurun_out/r5y_pipeline_units.md
timeout -k 10 200 python bench.py --model mlp --steps 30 --warmup 10 > gpurun_out/r5y_one.log 2>&1 || { tail -20 gpurun_out/r5y_one.log; exit 1; }
echo "mlp $(tail -1 gpurun_out/r5y_one.log | cut -c150-200)"
PDE_MLP_MEGA=0 timeout -k 10 200 python bench.py --model mlp --steps 30 --warmup 10 > gpurun_out/r5y_one.log 2>&1 || { tail -20 gpurun_out/r5y_one.log; exit 1; }
echo "mlp layerwise $(tail -1 gpurun_out/r5y_one.log | cut -c150-200)"
