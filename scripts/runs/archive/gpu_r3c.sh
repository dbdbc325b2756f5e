#!/bin/bash
# Round-3 profile C: hipGraph kernel traces (rocprofv3 --kernel-trace) of the ResNet-50 bench and of both
# pipeline stages at micro-batch 8 -> per-step kernel tables (scripts/graph_kernel_table.py).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run() {  # name, bench args...
  local name=$1; shift
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/tl_$name" -o "$name" --output-format csv \
    -- python3 "$R/bench.py" "$@" > "$R/gpurun_out/tl_$name.log" 2>&1 || { echo "trace $name failed"; tail -5 "$R/gpurun_out/tl_$name.log"; return 1; }
  cd "$R"
  f=$(find gpurun_out/tl_$name -name '*kernel_trace.csv' | head -1)
  tail -1 gpurun_out/tl_$name.log | cut -c1-400
  python3 scripts/graph_kernel_table.py "$f" --title "$name: hipGraph replay kernel trace" > gpurun_out/tl_$name.md
  head -14 gpurun_out/tl_$name.md
}
run mlp --model mlp --steps 40 --warmup 10 && \
run resnet50 --model resnet50 --steps 20 --warmup 10 && \
run stage1_m8 --model resnet50_stage --stage 1 --batch 8 --steps 30 --warmup 10 && \
run stage2_m8 --model resnet50_stage --stage 2 --batch 8 --steps 30 --warmup 10
