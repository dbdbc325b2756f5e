#!/bin/bash
# Round-4 check AM: P9 A operand from e1 words written by the P7b epilogue (dead mark in a1).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -k cnn -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r4am_pytest.log 2>&1 || { tail -30 gpurun_out/r4am_pytest.log; exit 1; }
tail -1 gpurun_out/r4am_pytest.log
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 > gpurun_out/r4am_one.log 2>&1 || { tail -20 gpurun_out/r4am_one.log; exit 1; }
  tail -1 gpurun_out/r4am_one.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'])"
done
timeout -k 10 120 python scripts/cnn_phase_stamps.py 2>&1 | grep -v amdgpu.ids | tail -6
