#!/bin/bash
# Round-6 S: full GPU suite + smoke + driver-config bench + ResNet-50 (low-K path at K <= 64).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r6s_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" gpurun_out/r6s_pytest.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6s_smoke.log 2>&1 || { tail -5 gpurun_out/r6s_smoke.log; exit 1; }
tail -2 gpurun_out/r6s_smoke.log
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6s_bench.log 2>&1 || { tail -5 gpurun_out/r6s_bench.log; exit 1; }
grep '^{' gpurun_out/r6s_bench.log | cut -c1-300
timeout -k 10 200 python bench.py --model resnet50 --steps 30 --warmup 10 > gpurun_out/r6s_resnet50.log 2>&1 || { tail -5 gpurun_out/r6s_resnet50.log; exit 1; }
grep '^{' gpurun_out/r6s_resnet50.log | cut -c1-200
