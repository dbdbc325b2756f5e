#!/bin/bash
# Round-6 J: config-4 rehearsal with both pipelines on the SAME batch (are the two pipelines deterministic twins?)
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for same in 1; do
  PIPE_DP_SAME_BATCH=$same timeout -k 10 300 python -u -m pytest "tests/test_pipeline_gpu.py::test_resnet_pipeline_x_dp_xgmi_graph_rehearsal_one_gpu[eager]" -s --timeout 200 --timeout-method thread > gpurun_out/r6j_same$same.log 2>&1
  echo "same=$same rc=$?"
  grep "PIPEDP losses" gpurun_out/r6j_same$same.log | head -1 | cut -c1-700
done
PDE_PIPE_MB_GROUP=1 timeout -k 10 300 python -u -m pytest "tests/test_pipeline_gpu.py::test_resnet_pipeline_x_dp_xgmi_graph_rehearsal_one_gpu[eager]" -s --timeout 200 --timeout-method thread > gpurun_out/r6j_g1.log 2>&1
echo "g1 rc=$?"; grep "PIPEDP losses" gpurun_out/r6j_g1.log | head -1 | cut -c1-700
