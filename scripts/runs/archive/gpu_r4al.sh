#!/bin/bash
# Round-4 check AL: conv1 bias gradient from the P9 MFMA (B column 25 = 1), DPP-gathered 16-byte stores.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -k cnn -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r4al_pytest.log 2>&1 || { tail -30 gpurun_out/r4al_pytest.log; exit 1; }
tail -1 gpurun_out/r4al_pytest.log
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 > gpurun_out/r4al_one.log 2>&1 || { tail -20 gpurun_out/r4al_one.log; exit 1; }
  tail -1 gpurun_out/r4al_one.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'])"
done
timeout -k 10 120 python scripts/cnn_phase_stamps.py 2>&1 | grep -v amdgpu.ids | tail -6
