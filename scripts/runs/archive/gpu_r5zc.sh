#!/bin/bash
# Round-5 ZC: pipeline stages without the zero fill -- pipeline tests, the re-measured unit table (g = 1/2/4),
# the ResNet-50 graph kernel table, and the world-2 resnet50_pp rehearsal on one GPU.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -m pytest -x -q --timeout 120 --timeout-method thread tests/test_pipeline_gpu.py tests/test_bnfold_gpu.py \
  > gpurun_out/r5zc_pytest.log 2>&1 || { tail -30 gpurun_out/r5zc_pytest.log; exit 1; }
tail -1 gpurun_out/r5zc_pytest.log
: > gpurun_out/r5zc_stages.jsonl
for g in 1 2 4; do for s in 1 2; do
  timeout -k 10 200 python bench.py --model resnet50_stage --stage $s --batch $((8 * g)) --mb-group $g --steps 30 --warmup 10 \
    > gpurun_out/r5zc_one.log 2>&1 || { tail -20 gpurun_out/r5zc_one.log; exit 1; }
  tail -1 gpurun_out/r5zc_one.log >> gpurun_out/r5zc_stages.jsonl
done; done
timeout -k 10 200 python bench.py --model resnet50 --steps 30 --warmup 10 > gpurun_out/r5zc_one.log 2>&1 || { tail -20 gpurun_out/r5zc_one.log; exit 1; }
tail -1 gpurun_out/r5zc_one.log > gpurun_out/r5zc_resnet50.jsonl
python3 scripts/pipeline_units.py gpurun_out/r5zc_stages.jsonl --one-gpu gpurun_out/r5zc_resnet50.jsonl --json gpurun_out/r5zc_pipeline_units.json \
  > gpurun_out/r5zc_pipeline_units.md && cat gpurun_out/r5zc_pipeline_units.md
bash scripts/gpu_rehearse_world2.sh resnet50_pp > gpurun_out/r5zc_world2.txt 2>&1 || { echo "world2 failed"; tail -20 gpurun_out/r5zc_world2.txt; exit 1; }
cut -c1-600 gpurun_out/r5zc_world2.txt | tail -3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r5zc_prof_r50" -o r50 --output-format csv -- python3 "$R/bench.py" \
  --model resnet50 --steps 40 --warmup 5 > "$R/gpurun_out/r5zc_prof_r50.log" 2>&1 || { echo "profile failed"; exit 1; }
python3 "$R/scripts/graph_kernel_table.py" "$R/gpurun_out/r5zc_prof_r50/r50_kernel_trace.csv" --title "resnet50 r5zc" --step-kernel k_optim \
  > "$R/gpurun_out/r5zc_resnet50_graph_kernels.md" && head -12 "$R/gpurun_out/r5zc_resnet50_graph_kernels.md"
