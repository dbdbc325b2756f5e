#!/bin/bash
# Round-6 AK: end-of-round kernel tables (graph mode): ResNet-50 b32 and the driver-config CNN step.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r6ak_r50" -o r --output-format csv -- python3 "$R/bench.py" \
    --model resnet50 --steps 40 --warmup 8 > "$R/gpurun_out/r6ak_r50.log" 2>&1 || { echo "profile failed"; exit 1; }
cd "$R"
python3 scripts/graph_kernel_table.py gpurun_out/r6ak_r50/r_kernel_trace.csv --title "resnet50 b32 graph r6ak" --step-kernel k_optim > gpurun_out/r6ak_resnet50_graph_kernels.md && head -26 gpurun_out/r6ak_resnet50_graph_kernels.md | cut -c1-150
