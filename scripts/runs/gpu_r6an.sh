#!/bin/bash
# Round-6 AN: post-revert sanity: BatchNorm / model numerics, smoke, driver-config bench.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6an_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/r6an_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6an_smoke.log 2>&1 || { tail -5 gpurun_out/r6an_smoke.log; exit 1; }
tail -1 gpurun_out/r6an_smoke.log
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6an_bench.log 2>&1 || { tail -5 gpurun_out/r6an_bench.log; exit 1; }
grep '^{' gpurun_out/r6an_bench.log | cut -c1-250
