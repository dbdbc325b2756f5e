#!/bin/bash
# GEMM shape tables (round-3 profile J): GEMM shape tables -- eager runs with PDE_GEMM_LOG=1 under rocprofv3 --kernel-trace, joined
# per launch by scripts/gemm_shape_table.py (resnet50 b32, stage 1 / 2 at a batch-32 unit, mlp).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1 PDE_GEMM_LOG=1 PDE_BENCH_PHASES=0
run() {  # name, bench args...
  local name=$1; shift
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/gs_$name" -o "$name" --output-format csv \
    -- python3 "$R/bench.py" --no-graph --steps 3 --warmup 1 "$@" > "$R/gpurun_out/gs_$name.log" 2>&1 || { echo "trace $name failed"; tail -5 "$R/gpurun_out/gs_$name.log"; return 1; }
  cd "$R"
  f=$(find gpurun_out/gs_$name -name '*kernel_trace.csv' | head -1)
  python3 scripts/gemm_shape_table.py gpurun_out/gs_$name.log "$f" --steps 4 --title "$name: GEMM launches of one eager step" > gpurun_out/gs_$name.md
  head -20 gpurun_out/gs_$name.md
}
run resnet50 --model resnet50 && run mlp --model mlp && \
run stage1_u32 --model resnet50_stage --stage 1 --batch 32 --mb-group 4 && \
run stage2_u32 --model resnet50_stage --stage 2 --batch 32 --mb-group 4
