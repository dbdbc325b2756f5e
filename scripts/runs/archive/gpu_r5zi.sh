#!/bin/bash
# Round-5 ZI: sanity of the rebuilt tree (MLP kernel back at v6) -- MLP / kernel tests, smoke, default bench, mlp bench.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mlp_mega_gpu.py tests/test_kernels_gpu.py \
  > gpurun_out/r5zi_pytest.log 2>&1 || { tail -30 gpurun_out/r5zi_pytest.log; exit 1; }
tail -1 gpurun_out/r5zi_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5zi_smoke.log 2>&1 || { tail -20 gpurun_out/r5zi_smoke.log; exit 1; }
tail -1 gpurun_out/r5zi_smoke.log
timeout -k 10 200 python bench.py > gpurun_out/r5zi_one.log 2>&1 || { tail -20 gpurun_out/r5zi_one.log; exit 1; }
tail -1 gpurun_out/r5zi_one.log | cut -c1-300
timeout -k 10 200 python bench.py --model mlp --steps 200 --warmup 20 > gpurun_out/r5zi_one.log 2>&1 || { tail -20 gpurun_out/r5zi_one.log; exit 1; }
tail -1 gpurun_out/r5zi_one.log | cut -c1-300
