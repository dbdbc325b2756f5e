#!/bin/bash
# Round-6 G: config-4 rehearsal (pp2 x dp2 on one GPU, xGMI DP communicator inside the captured step), two-shot
# tests, the Horovod-elastic step without the optimiser's unused layout refresh.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest "tests/test_pipeline_gpu.py::test_resnet_pipeline_x_dp_xgmi_graph_rehearsal_one_gpu" tests/test_xgmi_twoshot_gpu.py "tests/test_pipeline_gpu.py::test_resnet_pipeline_graph_rehearsal_one_gpu" "tests/test_elastic_gpu.py::test_hvd_elastic_script_survives_killed_worker_one_gpu" -x -v --timeout 300 --timeout-method thread > gpurun_out/r6g_pytest.log 2>&1 || { tail -40 gpurun_out/r6g_pytest.log; exit 1; }
tail -6 gpurun_out/r6g_pytest.log
cat gpurun_out/r6_world4_shared_gpu_resnet50_pp.jsonl
timeout -k 10 300 python bench.py --model hvd_cnn_elastic --steps 200 --warmup 20 > gpurun_out/r6g_hvde.jsonl 2> gpurun_out/r6g_hvde.err || { tail -20 gpurun_out/r6g_hvde.err; exit 1; }
cut -c1-400 gpurun_out/r6g_hvde.jsonl
