#!/bin/bash
# Generic A/B check of one switch: GPU tests (TESTS, default kernel + model + stream/pair tests), then bench.py
# for each model in MODELS with the switch at each value in VALUES.
#   AB_VAR=PDE_BN_SMALL VALUES="1 0" MODELS="resnet50" bash scripts/gpu_ab.sh
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TESTS=${TESTS:-tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_streams_gpu.py}
if [ "$TESTS" != "none" ]; then
  timeout -k 10 500 python -u -m pytest $TESTS -x -q --timeout 150 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
  rc=$?; grep -E "FAILED|Error|passed|failed" gpurun_out/ab_tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
fi
for m in ${MODELS:-resnet50 mlp}; do
  for v in ${VALUES:-1 0}; do
    env "$AB_VAR=$v" timeout -k 10 300 python bench.py --model $m --steps ${STEPS:-30} --warmup 10 ${BENCH_ARGS:-} > gpurun_out/ab_${m}_$v.log 2>&1 || { tail -5 gpurun_out/ab_${m}_$v.log; exit 1; }
    echo "$m $AB_VAR=$v: $(tail -1 gpurun_out/ab_${m}_$v.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], "img/s", r["ms_per_step"], "ms/step")')"
  done
done
