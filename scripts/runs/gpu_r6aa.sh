#!/bin/bash
# Round-6 AA: conv dgrad split-K slabs summed by the BatchNorm backward (no reduce launch): numerics + A/B benches.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_models_gpu.py tests/test_pipeline_gpu.py tests/test_kernels_gpu.py tests/test_streams_gpu.py tests/test_bnfold_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r6aa_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|Error|passed|failed" gpurun_out/r6aa_pytest.log | tail -5
[ $rc -eq 0 ] || exit $rc
bench() {  # label, args...
  local label=$1; shift
  timeout -k 10 200 python bench.py "$@" > gpurun_out/r6aa_$label.log 2>&1 || { tail -5 gpurun_out/r6aa_$label.log; return 1; }
  echo "$label $(grep '^{' gpurun_out/r6aa_$label.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"].get("final_loss"))')"
}
for rep in 1 2; do
  bench s2_on$rep --model resnet50_stage --stage 2 --batch 8 --steps 40 --warmup 5 || exit 1
  PDE_BN_BWD_DEFER=0 bench s2_off$rep --model resnet50_stage --stage 2 --batch 8 --steps 40 --warmup 5 || exit 1
done
bench s1_on --model resnet50_stage --stage 1 --batch 8 --steps 40 --warmup 5 || exit 1
PDE_BN_BWD_DEFER=0 bench s1_off --model resnet50_stage --stage 1 --batch 8 --steps 40 --warmup 5 || exit 1
bench r50_on --model resnet50 --steps 30 --warmup 10 || exit 1
PDE_BN_BWD_DEFER=0 bench r50_off --model resnet50 --steps 30 --warmup 10 || exit 1
