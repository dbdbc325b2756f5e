#!/bin/bash
# Round-4 check R: fused CNN -- P7b's B operand from registers (PDE_CNN_BREG=1) vs LDS, and a timing-only
# diagnostic that skips P1's fragment stores (PDE_CNN_DIAG_FRAG=1).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
PDE_CNN_BREG=1 timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -k cnn -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r4r_pytest.log 2>&1 || { tail -30 gpurun_out/r4r_pytest.log; exit 1; }
tail -1 gpurun_out/r4r_pytest.log
for cfg in "PDE_CNN_BREG=0" "PDE_CNN_BREG=1" "PDE_CNN_DIAG_FRAG=1"; do
  echo "== $cfg"
  env $cfg timeout -k 10 120 python scripts/cnn_phase_stamps.py > gpurun_out/r4r_stamps.txt 2>&1 || { tail -20 gpurun_out/r4r_stamps.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/r4r_stamps.txt
done
: > gpurun_out/r4r_bench.txt
for rep in 1 2 3; do for cfg in "PDE_CNN_BREG=0" "PDE_CNN_BREG=1"; do
  env $cfg timeout -k 10 200 python bench.py --steps 200 --warmup 20 > gpurun_out/r4r_one.log 2>&1 || { tail -20 gpurun_out/r4r_one.log; exit 1; }
  tail -1 gpurun_out/r4r_one.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', d['ms_per_step'], d['value'])" | tee -a gpurun_out/r4r_bench.txt
done; done
