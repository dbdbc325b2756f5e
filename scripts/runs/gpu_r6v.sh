#!/bin/bash
# Round-6 V: high-priority comm side streams (pipeline sends, overlapped RCCL): pipeline / comm / stream tests.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_pipeline_gpu.py tests/test_comm_gpu.py tests/test_streams_gpu.py tests/test_bn_sidestream_gpu.py tests/test_multigpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r6v_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|Error|passed|failed" gpurun_out/r6v_pytest.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model resnet50_pp --steps 20 --warmup 5 > gpurun_out/r6v_pp.log 2>&1 || { tail -5 gpurun_out/r6v_pp.log; exit 1; }
grep '^{' gpurun_out/r6v_pp.log | cut -c1-400
