#!/bin/bash
# Round-6 H: config-4 rehearsal, graph and eager forms (losses of both pipelines against one process).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest "tests/test_pipeline_gpu.py::test_resnet_pipeline_x_dp_xgmi_graph_rehearsal_one_gpu" -v -s --timeout 300 --timeout-method thread > gpurun_out/r6h_pytest.log 2>&1
echo "rc=$?"
grep "PIPEDP losses\|PASSED\|FAILED\|passed\|failed" gpurun_out/r6h_pytest.log | cut -c1-700
