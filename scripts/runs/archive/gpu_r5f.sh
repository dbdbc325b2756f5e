#!/bin/bash
# Round-5 F: GEMM launch tables of the m = 8 pipeline stages (eager, traced) under the ring core.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp PDE_GEMM_LOG=1 PDE_BENCH_PHASES=0 PDE_BENCH_OVERHEADS=0 PYTHONUNBUFFERED=1
mkdir -p "$R/gpurun_out"
for s in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r5f_gs_s$s" -o "r" --output-format csv \
    -- python3 "$R/bench.py" --no-graph --steps 3 --warmup 1 --model resnet50_stage --stage $s --batch 8 > "$R/gpurun_out/r5f_gs_s$s.log" 2>&1 || { echo "trace failed"; exit 1; }
  f=$(find "$R/gpurun_out/r5f_gs_s$s" -name '*kernel_trace.csv' | head -1)
  python3 "$R/scripts/gemm_shape_table.py" "$R/gpurun_out/r5f_gs_s$s.log" "$f" --steps 4 --title "stage $s m8 ring: GEMM launches of one eager step" > "$R/gpurun_out/r5f_gs_s$s.md"
  head -24 "$R/gpurun_out/r5f_gs_s$s.md"
done
