#!/bin/bash
# rocprofv3 kernel-trace + stats of bench.py for the given models (default: cnn mlp resnet50).
# Output: gpurun_out/prof_<model>/<model>_kernel_stats.csv ; summarise with scripts/prof_summary.py.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
models=${@:-cnn mlp resnet50}
for m in $models; do
  steps=20; [ "$m" = "resnet50" ] && steps=10
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$m" -o "$m" \
    --output-format csv -- python3 "$R/bench.py" --model "$m" --steps $steps --warmup 3 --no-graph \
    > "$R/gpurun_out/prof_$m.log" 2>&1 || { echo "profile $m failed"; tail -5 "$R/gpurun_out/prof_$m.log"; exit 1; }
  cd "$R" && python3 scripts/prof_summary.py "gpurun_out/prof_$m/${m}_kernel_stats.csv" $((steps + 6))
  python3 scripts/prof_summary.py "gpurun_out/prof_$m/${m}_kernel_stats.csv" $((steps + 6)) --md > "gpurun_out/prof_$m.md"
done
