#!/bin/bash
# One GPU round: every GPU test (per-test timeout), smoke, fused-CNN phase stamps, the three benches and
# rocprofv3 kernel statistics of the CNN and ResNet-50 benches.  Stops at the first GPU step that fails
# hard (timeout / abort / fault); test failures (rc 1) still let the benches run.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -60
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 120 python scripts/cnn_phase_stamps.py > gpurun_out/stamps.log 2>&1 || { tail -20 gpurun_out/stamps.log; exit 1; }
cat gpurun_out/stamps.log
for m in ${BENCH_MODELS:-cnn mlp resnet50}; do
  timeout -k 10 300 python bench.py --model $m --steps 30 --warmup 10 > gpurun_out/bench_$m.log 2>&1 || { tail -20 gpurun_out/bench_$m.log; exit 1; }
  tail -1 gpurun_out/bench_$m.log
done
[ "${PDE_PROFILE:-1}" = "1" ] || exit 0
bash scripts/gpu_profile.sh ${PROFILE_MODELS:-cnn resnet50}
