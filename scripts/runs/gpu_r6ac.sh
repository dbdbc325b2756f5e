#!/bin/bash
# Round-6 AC: stage kernel tables at m = 8 after the backward slab deferral.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for s in 1 2; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r6ac_prof_s$s" -o s$s --output-format csv -- python3 "$R/bench.py" \
    --model resnet50_stage --stage $s --batch 8 --steps 40 --warmup 5 > "$R/gpurun_out/r6ac_prof_s$s.log" 2>&1 || { echo "profile failed"; exit 1; }
  cd "$R"
  python3 scripts/graph_kernel_table.py gpurun_out/r6ac_prof_s$s/s${s}_kernel_trace.csv --title "resnet50 stage $s m8 r6ac" --step-kernel k_optim > gpurun_out/r6ac_stage${s}_m8_graph_kernels.md && head -24 gpurun_out/r6ac_stage${s}_m8_graph_kernels.md | cut -c1-150
done
