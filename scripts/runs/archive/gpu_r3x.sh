#!/bin/bash
# Round-3 check X: ResNet-50 hipGraph kernel trace with the all-finalize BatchNorm hand-off (per-call sequence).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/tl_r3x2" -o rn --output-format csv \
    -- python3 "$R/bench.py" --model resnet50 --steps 30 --warmup 10 > "$R/gpurun_out/tl_r3x2.log" 2>&1 || exit 1
cd "$R"; f=$(find gpurun_out/tl_r3x2 -name '*kernel_trace.csv' | head -1)
python3 scripts/graph_kernel_table.py "$f" --title "resnet50, all-finalize BatchNorm hand-off" > gpurun_out/r3x2_resnet50_graph_kernels.md; head -14 gpurun_out/r3x2_resnet50_graph_kernels.md
