#!/bin/bash
# Round-5 ZK: final-tree validation -- full GPU suite, smoke, default bench (driver config), model benches, ResNet trace.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r5zk_pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5zk_pytest.log | tail -8
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5zk_smoke.log 2>&1 || { tail -20 gpurun_out/r5zk_smoke.log; exit 1; }
tail -1 gpurun_out/r5zk_smoke.log
: > gpurun_out/r5zk_bench.jsonl
timeout -k 10 200 python bench.py > gpurun_out/r5zk_one.log 2>&1 && tail -1 gpurun_out/r5zk_one.log >> gpurun_out/r5zk_bench.jsonl
for m in "cnn" "hvd_cnn" "hvd_cnn_elastic" "mlp" "resnet50" "resnet50_stage --stage 1 --batch 8" "resnet50_stage --stage 2 --batch 8"; do
  timeout -k 10 200 python bench.py --model $m --steps 30 --warmup 10 > gpurun_out/r5zk_one.log 2>&1 || { tail -20 gpurun_out/r5zk_one.log; exit 1; }
  tail -1 gpurun_out/r5zk_one.log >> gpurun_out/r5zk_bench.jsonl
done
python - <<'PY'
import json
for l in open("gpurun_out/r5zk_bench.jsonl"):
    d = json.loads(l)
    print(d["config"]["model"], d["steps"], d["warmup"], d["ms_per_step"], d["value"])
PY
