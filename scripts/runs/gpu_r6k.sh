#!/bin/bash
# Round-6 K: config-4 rehearsal against a per-pipeline-copy single-process reference (graph + eager).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest "tests/test_pipeline_gpu.py::test_resnet_pipeline_x_dp_xgmi_graph_rehearsal_one_gpu" -s -v --timeout 240 --timeout-method thread > gpurun_out/r6k.log 2>&1
echo "rc=$?"
grep "PIPEDP losses\|PASSED\|FAILED" gpurun_out/r6k.log | cut -c1-700
