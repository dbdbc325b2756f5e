#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for fold in 1 0; do
  cd /tmp && PDE_MLP_FOLD_OPT=$fold timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/tl_mlpfold$fold" -o mlp --output-format csv \
    -- python3 "$R/bench.py" --model mlp --steps 40 --warmup 10 > "$R/gpurun_out/tl_mlpfold$fold.log" 2>&1 || exit 1
  cd "$R"
  f=$(find gpurun_out/tl_mlpfold$fold -name '*kernel_trace.csv' | head -1)
  python3 scripts/graph_kernel_table.py "$f" --title "mlp fold=$fold" > gpurun_out/tl_mlpfold$fold.md
  head -16 gpurun_out/tl_mlpfold$fold.md
done
