#!/bin/bash
# Round-6 D: pp2 x dp2 config-4 rehearsal (xGMI DP communicator, generous first-step wait), device-counter
# gather, elastic GPU tests (device commits), entry scripts (FusedHvdStep plain SGD).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest "tests/test_pipeline_gpu.py::test_resnet_pipeline_x_dp_xgmi_graph_rehearsal_one_gpu" tests/test_gather_counter_gpu.py tests/test_elastic_gpu.py -x -v --timeout 400 --timeout-method thread > gpurun_out/r6d_pytest.log 2>&1 || { tail -40 gpurun_out/r6d_pytest.log; exit 1; }
tail -8 gpurun_out/r6d_pytest.log
cat gpurun_out/r6_world4_shared_gpu_resnet50_pp.jsonl
timeout -k 10 600 python scripts/entry_scripts_measure.py gpurun_out/r6_entry_scripts.jsonl > gpurun_out/r6d_entry.log 2>&1 || { tail -40 gpurun_out/r6d_entry.log; exit 1; }
cat gpurun_out/r6d_entry.log
timeout -k 10 600 python bench.py --model elastic_cnn --gpus 2 --scale-to 1 --fault-at 300 --steps 100 --warmup 20 > gpurun_out/r6d_elastic_fault.jsonl 2> gpurun_out/r6d_elastic_fault.err || { tail -30 gpurun_out/r6d_elastic_fault.err; exit 1; }
tail -3 gpurun_out/r6d_elastic_fault.jsonl | cut -c1-1500
