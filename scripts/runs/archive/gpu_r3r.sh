#!/bin/bash
# Round-3 full check R: the whole GPU test suite, smoke(), and the benches of every model (+ stages, elastic
# world-1 round), saved for profiles/.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r3r_pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r3r_pytest.log | tail -12
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3r_smoke.log 2>&1 || { tail -20 gpurun_out/r3r_smoke.log; exit 1; }
tail -1 gpurun_out/r3r_smoke.log
: > gpurun_out/r3r_bench.jsonl
for m in "cnn" "mlp" "resnet50" "resnet50_stage --stage 1 --batch 8" "resnet50_stage --stage 2 --batch 8" \
         "resnet50_stage --stage 1 --batch 32 --mb-group 4" "resnet50_stage --stage 2 --batch 32 --mb-group 4"; do
  timeout -k 10 200 python bench.py --model $m --steps 30 --warmup 10 > gpurun_out/r3r_one.log 2>&1 || { tail -20 gpurun_out/r3r_one.log; exit 1; }
  tail -1 gpurun_out/r3r_one.log >> gpurun_out/r3r_bench.jsonl
  tail -1 gpurun_out/r3r_one.log | cut -c1-220
done
timeout -k 10 200 python bench.py > gpurun_out/r3r_default.log 2>&1 && tail -1 gpurun_out/r3r_default.log | cut -c1-300
