#!/bin/bash
# Fused-CNN iteration: model tests for the fused step, phase stamps, bench, and a rocprofv3 kernel profile
# of the graphed bench (graphs on: the timed configuration).
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=$(pwd)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -${TAILN:-12} "gpurun_out/$name.log"
  if [ $rc -gt 1 ]; then exit $rc; fi
  return 0
}
step cnn_tests 300 python -u -m pytest tests/test_models_gpu.py -k "cnn" -x -v --timeout 120 --timeout-method thread
step stamps 120 python scripts/cnn_phase_stamps.py
step bench_cnn 200 python bench.py --steps 50 --warmup 10
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_cnn" -o cnn --output-format csv \
  -- python3 "$R/bench.py" --steps 40 --warmup 5 > "$R/gpurun_out/prof_cnn.log" 2>&1 || { echo "profile failed"; tail -5 "$R/gpurun_out/prof_cnn.log"; exit 1; }
cd "$R" && python3 scripts/prof_summary.py gpurun_out/prof_cnn/cnn_kernel_stats.csv 45 --md | tee gpurun_out/prof_cnn.md | head -12
