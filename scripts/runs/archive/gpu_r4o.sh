#!/bin/bash
# Round-4 check O: DDP gradient views aligned to 256 B (the fused optimiser's vector path) -- model / DDP tests,
# MLP / ResNet-50 / CNN benches.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_models_gpu.py tests/test_comm_gpu.py tests/test_kernels_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r4o_pytest.log 2>&1 || { tail -30 gpurun_out/r4o_pytest.log; exit 1; }
tail -1 gpurun_out/r4o_pytest.log
: > gpurun_out/r4o_bench.jsonl
for m in mlp resnet50 cnn mlp; do
  timeout -k 10 200 python bench.py --model $m --steps 50 --warmup 10 > gpurun_out/r4o_one.log 2>&1 || { tail -20 gpurun_out/r4o_one.log; exit 1; }
  tail -1 gpurun_out/r4o_one.log >> gpurun_out/r4o_bench.jsonl
  python -c "import json; d=json.loads(open('gpurun_out/r4o_one.log').read().strip().splitlines()[-1]); print(d['config']['model'], d['ms_per_step'], d['value'], d['config'].get('phases'))"
done
