#!/bin/bash
# GPU check: all GPU tests, smoke, benches (cnn/mlp/resnet50), rocprof kernel stats of the default bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc   # 1 = test failures: still run smoke/bench
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
for m in cnn mlp resnet50; do
  timeout -k 10 300 python bench.py --model $m --steps 30 --warmup 10 > gpurun_out/bench_$m.log 2>&1 || { tail -20 gpurun_out/bench_$m.log; exit 1; }
  tail -1 gpurun_out/bench_$m.log
done
[ "${PDE_PROFILE:-1}" = "1" ] || exit 0
bash scripts/gpu_profile.sh cnn resnet50
