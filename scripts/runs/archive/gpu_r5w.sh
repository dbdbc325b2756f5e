#!/bin/bash
# Round-5 W: final validation -- full GPU suite, smoke, default bench (driver config), model benches, ResNet trace.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r5w_pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5w_pytest.log | tail -8
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5w_smoke.log 2>&1 || { tail -20 gpurun_out/r5w_smoke.log; exit 1; }
tail -1 gpurun_out/r5w_smoke.log
: > gpurun_out/r5w_bench.jsonl
timeout -k 10 200 python bench.py > gpurun_out/r5w_one.log 2>&1 && tail -1 gpurun_out/r5w_one.log >> gpurun_out/r5w_bench.jsonl
for m in "cnn" "hvd_cnn" "hvd_cnn_elastic" "mlp" "resnet50" "resnet50_stage --stage 1 --batch 8" "resnet50_stage --stage 2 --batch 8"; do
  timeout -k 10 200 python bench.py --model $m --steps 30 --warmup 10 > gpurun_out/r5w_one.log 2>&1 || { tail -20 gpurun_out/r5w_one.log; exit 1; }
  tail -1 gpurun_out/r5w_one.log >> gpurun_out/r5w_bench.jsonl
done
python - <<'PY'
import json
for l in open("gpurun_out/r5w_bench.jsonl"):
    d = json.loads(l)
    print(d["config"]["model"], d["steps"], d["warmup"], d["ms_per_step"], d["value"])
PY
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r5w_prof_r50" -o r50 --output-format csv -- python3 "$R/bench.py" \
  --model resnet50 --steps 40 --warmup 5 > "$R/gpurun_out/r5w_prof_r50.log" 2>&1 || { echo "profile failed"; exit 1; }
python3 "$R/scripts/graph_kernel_table.py" "$R/gpurun_out/r5w_prof_r50/r50_kernel_trace.csv" --title "resnet50 r5w" --step-kernel k_optim \
  > "$R/gpurun_out/r5w_resnet50_graph_kernels.md" && head -16 "$R/gpurun_out/r5w_resnet50_graph_kernels.md"
