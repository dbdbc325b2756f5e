#!/bin/bash
# Round-6 C: two-shot xGMI all-reduce (2/4 ranks on one GPU), pp2 x dp2 config-4 rehearsal with the xGMI DP
# communicator inside the captured step, entry scripts again (FusedHvdStep plain-SGD path).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_xgmi_twoshot_gpu.py tests/test_xgmi_gpu.py "tests/test_pipeline_gpu.py::test_resnet_pipeline_x_dp_xgmi_graph_rehearsal_one_gpu" tests/test_entry_fast_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r6c_pytest.log 2>&1 || { tail -40 gpurun_out/r6c_pytest.log; exit 1; }
tail -12 gpurun_out/r6c_pytest.log
cat gpurun_out/r6_world4_shared_gpu_resnet50_pp.jsonl
timeout -k 10 600 python scripts/entry_scripts_measure.py gpurun_out/r6_entry_scripts.jsonl > gpurun_out/r6c_entry.log 2>&1 || { tail -40 gpurun_out/r6c_entry.log; exit 1; }
cat gpurun_out/r6c_entry.log
