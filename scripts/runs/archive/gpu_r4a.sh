#!/bin/bash
# Round-4 check A (session start): benches of every model + the ResNet-50 hipGraph kernel table, to re-baseline
# this round's box before any change.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
: > gpurun_out/r4a_bench.jsonl
for m in "cnn" "mlp" "resnet50" "resnet50_stage --stage 1 --batch 8" "resnet50_stage --stage 2 --batch 8"; do
  timeout -k 10 200 python bench.py --model $m --steps 30 --warmup 10 > gpurun_out/r4a_one.log 2>&1 || { tail -20 gpurun_out/r4a_one.log; exit 1; }
  tail -1 gpurun_out/r4a_one.log >> gpurun_out/r4a_bench.jsonl
  tail -1 gpurun_out/r4a_one.log | cut -c1-200
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/tl_r4a" -o rn --output-format csv \
    -- python3 "$R/bench.py" --model resnet50 --steps 30 --warmup 10 > "$R/gpurun_out/tl_r4a.log" 2>&1 || exit 1
cd "$R"; f=$(find gpurun_out/tl_r4a -name '*kernel_trace.csv' | head -1)
python3 scripts/graph_kernel_table.py "$f" --title "resnet50 r4a baseline" > gpurun_out/r4a_resnet50_graph_kernels.md; head -40 gpurun_out/r4a_resnet50_graph_kernels.md
