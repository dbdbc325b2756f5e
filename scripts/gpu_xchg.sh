#!/bin/bash
# xGMI exchange folded into the fused CNN reduction: rehearsal tests (2 and 4 ranks on one GPU), the fused
# CNN model tests, the 1-GPU headline bench (no regression at world 1).
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_xgmi_gpu.py tests/test_models_gpu.py tests/test_comm_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/xchg_tests.log 2>&1
rc=$?; grep -E "passed|failed|error|PASS|FAIL" gpurun_out/xchg_tests.log | tail -30; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/xchg_bench_cnn.log 2>&1 || { tail -5 gpurun_out/xchg_bench_cnn.log; exit 1; }
tail -1 gpurun_out/xchg_bench_cnn.log
