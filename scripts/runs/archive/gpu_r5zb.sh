#!/bin/bash
# Round-5 ZB: DDP(static_graph) skips the flat-gradient zero fill once every first writer stores (BatchNorm
# finalize and linear bias now first-write aware); persistent unit loss gradient -- numerics, ResNet-50 benches and
# a kernel trace of the ResNet-50 step (no ATen fill left).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_models_gpu.py \
  tests/test_bn_sidestream_gpu.py tests/test_bnfold_gpu.py tests/test_pipeline_gpu.py tests/test_streams_gpu.py \
  > gpurun_out/r5zb_pytest.log 2>&1 || { tail -30 gpurun_out/r5zb_pytest.log; exit 1; }
tail -1 gpurun_out/r5zb_pytest.log
: > gpurun_out/r5zb_bench.jsonl
for m in "resnet50" "resnet50_stage --stage 1 --batch 32 --mb-group 4" "resnet50_stage --stage 2 --batch 32 --mb-group 4" "resnet50_stage --stage 1 --batch 8" "resnet50_stage --stage 2 --batch 8" "resnet50"; do
  timeout -k 10 200 python bench.py --model $m --steps 30 --warmup 10 > gpurun_out/r5zb_one.log 2>&1 || { tail -20 gpurun_out/r5zb_one.log; exit 1; }
  tail -1 gpurun_out/r5zb_one.log >> gpurun_out/r5zb_bench.jsonl
  echo "$m $(tail -1 gpurun_out/r5zb_one.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r5zb_prof" -o run -- python "$R/bench.py" --model resnet50 --steps 200 --warmup 10 \
  > "$R/gpurun_out/r5zb_prof.log" 2>&1 || { tail -20 "$R/gpurun_out/r5zb_prof.log"; exit 1; }
cd "$R"
f=$(find gpurun_out/r5zb_prof -name "*kernel_stats.csv" | head -1)
echo "stats: $f"; grep -c "" "$f"; grep -i "fill" "$f" || echo "no fill kernels"
