#!/bin/bash
# Round-4 check U: fused CNN with bf16 activation columns for the fc1 weight gradient.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -k cnn -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r4u_pytest.log 2>&1 || { tail -30 gpurun_out/r4u_pytest.log; exit 1; }
tail -1 gpurun_out/r4u_pytest.log
timeout -k 10 120 python scripts/cnn_phase_stamps.py > gpurun_out/r4u_stamps.txt 2>&1 || { tail -20 gpurun_out/r4u_stamps.txt; exit 1; }
cat gpurun_out/r4u_stamps.txt
for i in 1 2 3; do
timeout -k 10 200 python bench.py --steps 200 --warmup 20 > gpurun_out/r4u_one.log 2>&1 || { tail -20 gpurun_out/r4u_one.log; exit 1; }
tail -1 gpurun_out/r4u_one.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'])"
done
for d in 1 4 8 0; do
  PDE_CNN_DIAG=$d timeout -k 10 200 python bench.py --steps 200 --warmup 20 > gpurun_out/r4u_one.log 2>&1 || { tail -20 gpurun_out/r4u_one.log; exit 1; }
  tail -1 gpurun_out/r4u_one.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('diag=$d', d['ms_per_step'], d['value'])"
done
