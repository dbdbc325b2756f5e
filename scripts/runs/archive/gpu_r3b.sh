#!/bin/bash
# Round-3 check B: parameter-server ring data plane, hybrid script, elastic rehearsal, then benches
# (cnn / resnet50 / stage 1 and 2 at micro-batch 8) with their phase timers.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_pipeline_gpu.py tests/test_elastic_gpu.py -v --timeout 300 \
  --timeout-method thread -k "parameter_server or hybrid or elastic" 2>&1 | tee gpurun_out/r3b_pytest.log
rc=${PIPESTATUS[0]}
[ $rc -le 1 ] || exit $rc
for m in "cnn" "resnet50" "resnet50_stage --stage 1 --batch 8" "resnet50_stage --stage 2 --batch 8"; do
  timeout -k 10 200 python bench.py --model $m --steps 30 --warmup 10 2>&1 | tee -a gpurun_out/r3b_bench.log | tail -1 || exit 1
done
