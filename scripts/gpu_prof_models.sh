#!/bin/bash
# rocprofv3 kernel statistics of the graphed bench for the given models (the timed configuration), plus the
# plain bench lines.  Usage: gpu_prof_models.sh [tag] [models...]
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=$(pwd)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
tag=${1:-r2}; shift
models=${@:-mlp resnet50}
for m in $models; do
  steps=40; [ "$m" = "resnet50" ] && steps=20
  timeout -k 10 300 python bench.py --model $m --steps $steps --warmup 10 > gpurun_out/bench_${tag}_$m.log 2>&1 || { tail -5 gpurun_out/bench_${tag}_$m.log; exit 1; }
  tail -1 gpurun_out/bench_${tag}_$m.log
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${tag}_$m" -o "$m" --output-format csv \
    -- python3 "$R/bench.py" --model "$m" --steps $steps --warmup 5 > "$R/gpurun_out/prof_${tag}_$m.log" 2>&1 || { echo "profile $m failed"; tail -5 "$R/gpurun_out/prof_${tag}_$m.log"; exit 1; }
  cd "$R"
  python3 scripts/prof_summary.py gpurun_out/prof_${tag}_$m/${m}_kernel_stats.csv $((steps + 9)) --md > gpurun_out/prof_${tag}_$m.md
  head -24 gpurun_out/prof_${tag}_$m.md
done
