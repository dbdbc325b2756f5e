#!/bin/bash
# Round-4 check C: Horovod path -- hvd_cnn at world 1 (vs the DDP headline) and the world-2 one-GPU rehearsal
# (xGMI one-shot data plane, response cache, graph mode); comm tests.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_comm_gpu.py -m gpu -v -x --timeout 300 --timeout-method thread > gpurun_out/r4c_pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r4c_pytest.log | tail -12
[ $rc -eq 0 ] || { tail -40 gpurun_out/r4c_pytest.log; exit $rc; }
: > gpurun_out/r4c_bench.jsonl
for m in cnn hvd_cnn cnn hvd_cnn mlp resnet50; do
  timeout -k 10 200 python bench.py --model $m --steps 100 --warmup 20 > gpurun_out/r4c_one.log 2>&1 || { tail -20 gpurun_out/r4c_one.log; exit 1; }
  tail -1 gpurun_out/r4c_one.log >> gpurun_out/r4c_bench.jsonl
  tail -1 gpurun_out/r4c_one.log | cut -c1-200
done
