#!/bin/bash
# Round-4 check K: fused-CNN output stores (PDE_CNN_STORE 0 plain / 1 nt / 2 sc1 write-through) x XCD-aware
# image mapping (PDE_CNN_XMAP), plus the fused-CNN model tests.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -k cnn -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r4k_pytest.log 2>&1 || { tail -30 gpurun_out/r4k_pytest.log; exit 1; }
tail -1 gpurun_out/r4k_pytest.log
: > gpurun_out/r4k_bench.txt
for rep in 1 2; do
for cfg in "PDE_CNN_XMAP=0 PDE_CNN_STORE=0" "PDE_CNN_XMAP=1 PDE_CNN_STORE=0" "PDE_CNN_XMAP=0 PDE_CNN_STORE=1" "PDE_CNN_XMAP=1 PDE_CNN_STORE=1" "PDE_CNN_XMAP=0 PDE_CNN_STORE=2" "PDE_CNN_XMAP=1 PDE_CNN_STORE=2"; do
  env $cfg timeout -k 10 200 python bench.py --steps 200 --warmup 20 > gpurun_out/r4k_one.log 2>&1 || { tail -20 gpurun_out/r4k_one.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4k_one.log').read().strip().splitlines()[-1]); print('$cfg', d['ms_per_step'], d['value'], d['config']['final_loss'])" | tee -a gpurun_out/r4k_bench.txt
done
done
for cfg in "PDE_CNN_XMAP=1 PDE_CNN_STORE=0 PDE_CNN_DIAG=1" "PDE_CNN_XMAP=1 PDE_CNN_STORE=2 PDE_CNN_DIAG=1"; do
  env $cfg timeout -k 10 200 python bench.py --steps 200 --warmup 20 > gpurun_out/r4k_one.log 2>&1 || { tail -20 gpurun_out/r4k_one.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4k_one.log').read().strip().splitlines()[-1]); print('$cfg', d['ms_per_step'], d['value'])" | tee -a gpurun_out/r4k_bench.txt
done
