#!/bin/bash
# Round-3 check D: full GPU test suite; benches (cnn / mlp / resnet50 / stages at micro-batch 4, 8, 32, phase
# timers); hipGraph kernel tables of mlp, resnet50 and both stages (scripts/runs/archive/gpu_r3c.sh).
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/r3d_pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r3d_pytest.log | tail -30
[ $rc -le 1 ] || exit $rc
: > gpurun_out/r3d_bench.jsonl
for m in "cnn" "mlp" "resnet50" "resnet50_stage --stage 1 --batch 8" "resnet50_stage --stage 2 --batch 8" \
         "resnet50_stage --stage 1 --batch 4" "resnet50_stage --stage 2 --batch 4" \
         "resnet50_stage --stage 1 --batch 32" "resnet50_stage --stage 2 --batch 32"; do
  timeout -k 10 200 python bench.py --model $m --steps 30 --warmup 10 > gpurun_out/r3d_bench_one.log 2>&1 || { tail -20 gpurun_out/r3d_bench_one.log; exit 1; }
  tail -1 gpurun_out/r3d_bench_one.log >> gpurun_out/r3d_bench.jsonl
  tail -1 gpurun_out/r3d_bench_one.log | cut -c1-240
done
bash scripts/runs/archive/gpu_r3c.sh
