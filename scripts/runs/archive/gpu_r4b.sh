#!/bin/bash
# Round-4 check B: elastic failure rehearsal on the fused/xGMI path (kill a worker mid-round), the xGMI + BN
# tests after the fail-fast / occupancy-cap changes, and the default bench.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_elastic_gpu.py tests/test_xgmi_gpu.py tests/test_kernels_gpu.py -m gpu -v -x \
    --timeout 300 --timeout-method thread > gpurun_out/r4b_pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r4b_pytest.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py > gpurun_out/r4b_default.log 2>&1 && tail -1 gpurun_out/r4b_default.log | cut -c1-300
