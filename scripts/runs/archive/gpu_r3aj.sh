#!/bin/bash
# Round-3 check AJ: MLP hipGraph kernel trace (per-step kernel table + one step's sequence).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/tl_r3aj" -o mlp --output-format csv \
    -- python3 "$R/bench.py" --model mlp --steps 60 --warmup 10 > "$R/gpurun_out/tl_r3aj.log" 2>&1 || exit 1
cd "$R"; f=$(find gpurun_out/tl_r3aj -name '*kernel_trace.csv' | head -1)
python3 scripts/graph_kernel_table.py "$f" --title "mlp" > gpurun_out/r3aj_mlp_graph_kernels.md; cat gpurun_out/r3aj_mlp_graph_kernels.md
python3 scripts/timeline_gaps.py "$f" --last 400 --seq 20 > gpurun_out/r3aj_mlp_timeline.txt; cat gpurun_out/r3aj_mlp_timeline.txt
