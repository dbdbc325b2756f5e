#!/bin/bash
# Round-4 check W: fused CNN with the conv2-weight slab block transposed (16-byte P7a stores) -- tests, stamps,
# store flavour A/B, hvd_cnn at world 1.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py tests/test_comm_gpu.py -k "cnn or hvd" -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r4w_pytest.log 2>&1 || { tail -30 gpurun_out/r4w_pytest.log; exit 1; }
tail -1 gpurun_out/r4w_pytest.log
timeout -k 10 120 python scripts/cnn_phase_stamps.py > gpurun_out/r4w_stamps.txt 2>&1 || { tail -20 gpurun_out/r4w_stamps.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r4w_stamps.txt
: > gpurun_out/r4w_bench.txt
for rep in 1 2; do for cfg in "PDE_CNN_STORE=2" "PDE_CNN_STORE=1" "PDE_CNN_STORE=0"; do
  env $cfg timeout -k 10 200 python bench.py --steps 200 --warmup 20 > gpurun_out/r4w_one.log 2>&1 || { tail -20 gpurun_out/r4w_one.log; exit 1; }
  tail -1 gpurun_out/r4w_one.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', d['ms_per_step'], d['value'])" | tee -a gpurun_out/r4w_bench.txt
done; done
timeout -k 10 200 python bench.py --model hvd_cnn --steps 200 --warmup 20 > gpurun_out/r4w_one.log 2>&1 || { tail -20 gpurun_out/r4w_one.log; exit 1; }
tail -1 gpurun_out/r4w_one.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('hvd_cnn', d['ms_per_step'], d['value'], d['config'].get('engine'))" | tee -a gpurun_out/r4w_bench.txt
