#!/bin/bash
# Round-5 R: split-K slab reduction with 4 loads in flight per lane -- numerics + ResNet / stage / MLP benches and
# a ResNet-50 graph kernel trace.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_streams_gpu.py > gpurun_out/r5r_pytest.log 2>&1 || { tail -20 gpurun_out/r5r_pytest.log; exit 1; }
tail -1 gpurun_out/r5r_pytest.log
: > gpurun_out/r5r_bench.jsonl
for m in "resnet50" "resnet50_stage --stage 1 --batch 8" "resnet50_stage --stage 2 --batch 8" "resnet50_stage --stage 1 --batch 32 --mb-group 4" "resnet50_stage --stage 2 --batch 32 --mb-group 4" "resnet50" "mlp"; do
  timeout -k 10 200 python bench.py --model $m --steps 30 --warmup 10 > gpurun_out/r5r_one.log 2>&1 || { tail -20 gpurun_out/r5r_one.log; exit 1; }
  tail -1 gpurun_out/r5r_one.log >> gpurun_out/r5r_bench.jsonl
  echo "$m | $(tail -1 gpurun_out/r5r_one.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r5r_prof_r50" -o r50 --output-format csv -- python3 "$R/bench.py" \
  --model resnet50 --steps 40 --warmup 5 > "$R/gpurun_out/r5r_prof_r50.log" 2>&1 || { echo "profile failed"; exit 1; }
python3 "$R/scripts/graph_kernel_table.py" "$R/gpurun_out/r5r_prof_r50/r50_kernel_trace.csv" --title "resnet50 r5r" --step-kernel k_optim \
  > "$R/gpurun_out/r5r_resnet50_graph_kernels.md" && head -30 "$R/gpurun_out/r5r_resnet50_graph_kernels.md"
