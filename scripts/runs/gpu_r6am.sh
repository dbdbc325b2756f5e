#!/bin/bash
# Round-6 AM: BatchNorm backward keeps the masked gradient in registers (no second y load): numerics + benches.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_pipeline_gpu.py tests/test_bnfold_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6am_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/r6am_pytest.log
[ $rc -eq 0 ] || exit $rc
bench() {  # label, args...
  local label=$1; shift
  timeout -k 10 200 python bench.py "$@" > gpurun_out/r6am_$label.log 2>&1 || { tail -5 gpurun_out/r6am_$label.log; return 1; }
  echo "$label $(grep '^{' gpurun_out/r6am_$label.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
}
for rep in 1 2; do
  bench r50_$rep --model resnet50 --steps 30 --warmup 10 || exit 1
  bench s1_$rep --model resnet50_stage --stage 1 --batch 8 --steps 40 --warmup 5 || exit 1
  bench s2_$rep --model resnet50_stage --stage 2 --batch 8 --steps 40 --warmup 5 || exit 1
done
