#!/bin/bash
# Round-6 L: fused AdamW for the Horovod-elastic CNN step (numerics + elastic kill test + bench), and the config-4
# rehearsal against per-pipeline-copy references (graph + eager).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -k "adamw or fused" -v --timeout 120 --timeout-method thread > gpurun_out/r6l_adamw.log 2>&1
rc=$?; echo "adamw rc=$rc"; grep "PASSED\|FAILED\|Error" gpurun_out/r6l_adamw.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --model hvd_cnn_elastic --steps 300 --warmup 30 > gpurun_out/r6l_bench_hvd_elastic.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/r6l_bench_hvd_elastic.log | cut -c1-1500
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_elastic_gpu.py -k hvd -v --timeout 240 --timeout-method thread > gpurun_out/r6l_elastic.log 2>&1
rc=$?; echo "elastic rc=$rc"; grep "PASSED\|FAILED" gpurun_out/r6l_elastic.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest "tests/test_pipeline_gpu.py::test_resnet_pipeline_x_dp_xgmi_graph_rehearsal_one_gpu" -s -v --timeout 240 --timeout-method thread > gpurun_out/r6l_ppdp.log 2>&1
echo "ppdp rc=$?"
grep "PIPEDP losses\|PASSED\|FAILED" gpurun_out/r6l_ppdp.log | cut -c1-700
