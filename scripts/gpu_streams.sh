#!/bin/bash
# Paired dgrad+wgrad check: stream/pair tests + model tests, then ResNet-50 / MLP benches with GEMM pairing
# on and off (PDE_GEMM_PAIR=0).
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_streams_gpu.py tests/test_models_gpu.py -v -x --timeout 120 --timeout-method thread > gpurun_out/pytest_streams.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|Error" gpurun_out/pytest_streams.log | tail -30
[ $rc -eq 0 ] || exit $rc
for m in ${MODELS:-resnet50 mlp}; do
  for s in 1 0; do
    PDE_GEMM_PAIR=$s timeout -k 10 300 python bench.py --model $m --steps 30 --warmup 10 > gpurun_out/bench_${m}_s$s.log 2>&1 || { tail -20 gpurun_out/bench_${m}_s$s.log; exit 1; }
    echo "gemm_pair=$s $(tail -1 gpurun_out/bench_${m}_s$s.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["model"], d["value"], d["ms_per_step"])')"
  done
done
