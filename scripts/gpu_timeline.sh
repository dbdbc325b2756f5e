#!/bin/bash
# rocprofv3 kernel trace of the hipGraph bench (the production path): per-step kernel sequence and idle gaps.
# Usage: bash scripts/gpu_timeline.sh [models...]   (default: cnn resnet50)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for m in ${@:-cnn resnet50}; do
  steps=40; seq=12; [ "$m" = "resnet50" ] && { steps=20; seq=0; }
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/tl_$m" -o "$m" \
    --output-format csv -- python3 "$R/bench.py" --model "$m" --steps $steps --warmup 10 \
    > "$R/gpurun_out/tl_$m.log" 2>&1 || { echo "trace $m failed"; tail -5 "$R/gpurun_out/tl_$m.log"; exit 1; }
  cd "$R"
  f=$(ls gpurun_out/tl_$m/${m}_kernel_trace.csv 2>/dev/null || find gpurun_out/tl_$m -name '*kernel_trace.csv' | head -1)
  n=$(python3 -c "import csv,sys; print(sum(1 for _ in csv.DictReader(open('$f'))))")
  echo "== $m ($n kernels traced)"; tail -1 gpurun_out/tl_$m.log | cut -c1-200
  python3 scripts/timeline_gaps.py "$f" --last $((n / 3)) --seq $seq | tee gpurun_out/tl_$m.txt
done
