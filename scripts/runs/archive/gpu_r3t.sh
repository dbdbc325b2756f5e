#!/bin/bash
# Round-3 trace T: resnet50 hipGraph kernel traces with the BatchNorm chunk cap at 64 (default) and 256, for a
# per-grid comparison of the BatchNorm kernels (scripts/bn_grid_table.py).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for ch in 64 256; do
  cd /tmp && PDE_BN_CHUNKS=$ch timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/bn_ch$ch" -o r --output-format csv \
    -- python3 "$R/bench.py" --model resnet50 --steps 20 --warmup 5 > "$R/gpurun_out/bn_ch$ch.log" 2>&1 || exit 1
  cd "$R"; tail -1 gpurun_out/bn_ch$ch.log | cut -c1-160
done
