#!/bin/bash
# Round-6 AQ: entry-script and bench sanity after the data-plane change.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_entry_fast_gpu.py tests/test_comm_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r6aq_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/r6aq_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6aq_bench.log 2>&1 || { tail -5 gpurun_out/r6aq_bench.log; exit 1; }
grep '^{' gpurun_out/r6aq_bench.log | cut -c1-220
