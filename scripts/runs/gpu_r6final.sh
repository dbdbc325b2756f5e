#!/bin/bash
# Round-6 final: full GPU suite, smoke, driver-config bench, model benches (evidence for the round summary).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/final_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" gpurun_out/final_pytest.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { tail -5 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
for m in "--gpus 1 --steps 20 --warmup 5" "--model mlp --steps 100 --warmup 20" "--model hvd_cnn --steps 100 --warmup 20" "--model hvd_cnn_elastic --steps 300 --warmup 30" "--model resnet50 --steps 30 --warmup 10" "--model resnet50_stage --stage 1 --batch 8 --steps 40 --warmup 5" "--model resnet50_stage --stage 2 --batch 8 --steps 40 --warmup 5" "--steps 500 --warmup 50"; do
  timeout -k 10 200 python bench.py $m > gpurun_out/final_bench.log 2>&1 || { tail -5 gpurun_out/final_bench.log; exit 1; }
  grep '^{' gpurun_out/final_bench.log | tail -1 >> gpurun_out/final_bench.jsonl
  echo "$m -> $(grep '^{' gpurun_out/final_bench.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
