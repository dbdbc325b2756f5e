#!/bin/bash
# Round-5 ZN: kernel tables of the two pipeline stages at the default unit (g = 4), for the BatchNorm-fold work.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p "$R/gpurun_out"
for s in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r5zn_prof_s$s" -o s$s --output-format csv -- python3 "$R/bench.py" \
    --model resnet50_stage --stage $s --batch 32 --mb-group 4 --steps 40 --warmup 5 > "$R/gpurun_out/r5zn_prof_s$s.log" 2>&1 || { echo "profile failed"; tail -5 "$R/gpurun_out/r5zn_prof_s$s.log"; exit 1; }
  python3 "$R/scripts/graph_kernel_table.py" "$R/gpurun_out/r5zn_prof_s$s/s${s}_kernel_trace.csv" --title "resnet50 stage $s g4 r5zn" --step-kernel k_optim \
    > "$R/gpurun_out/r5zn_stage${s}_g4_graph_kernels.md" && head -12 "$R/gpurun_out/r5zn_stage${s}_g4_graph_kernels.md"
done
