#!/bin/bash
# Round-6 I: config-4 rehearsal numerics A/B -- the DP all-reduce over gloo (host) vs xGMI, eager split steps.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for comm in gloo xgmi; do
  PDE_PIPE_DP_COMM=$comm timeout -k 10 300 python -u -m pytest "tests/test_pipeline_gpu.py::test_resnet_pipeline_x_dp_xgmi_graph_rehearsal_one_gpu[eager]" -s --timeout 200 --timeout-method thread > gpurun_out/r6i_$comm.log 2>&1
  echo "$comm rc=$?"
  grep "PIPEDP losses" gpurun_out/r6i_$comm.log | head -1 | cut -c1-600
done
timeout -k 10 400 python -u -m pytest "tests/test_pipeline_gpu.py::test_resnet_pipeline_graph_rehearsal_one_gpu" -q --timeout 200 --timeout-method thread > gpurun_out/r6i_pp2.log 2>&1
echo "pp2 rc=$?"; tail -1 gpurun_out/r6i_pp2.log
