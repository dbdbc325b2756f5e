#!/bin/bash
# Round-4 check AJ: the single-launch fused CNN step (PDE_CNN_FUSED_TAIL=1, grid barrier) re-measured now that
# the slab / activation stores are write-through (the barrier's release has little left to write back).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
PDE_CNN_FUSED_TAIL=1 timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -k "fused_cnn" -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r4aj_pytest.log 2>&1 || { tail -30 gpurun_out/r4aj_pytest.log; exit 1; }
tail -1 gpurun_out/r4aj_pytest.log
for cfg in "PDE_X=0" "PDE_CNN_FUSED_TAIL=1" "PDE_X=0" "PDE_CNN_FUSED_TAIL=1"; do
  env $cfg timeout -k 10 200 python bench.py --steps 300 --warmup 20 > gpurun_out/r4aj_one.log 2>&1 || { tail -20 gpurun_out/r4aj_one.log; exit 1; }
  tail -1 gpurun_out/r4aj_one.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', d['ms_per_step'], d['value'])"
done
