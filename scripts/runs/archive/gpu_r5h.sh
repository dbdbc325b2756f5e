#!/bin/bash
# Round-5 H: the one-launch MLP step -- numerics tests, bench (driver config), kernel trace.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m pytest -x -v --timeout 120 --timeout-method thread tests/test_mlp_mega_gpu.py > gpurun_out/r5h_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|error|assert|passed|failed" gpurun_out/r5h_pytest.log | head -30
[ $rc -eq 0 ] || exit $rc
for cfg in "PDE_MLP_MEGA=0" "PDE_MLP_MEGA=1"; do
  env $cfg timeout -k 10 200 python bench.py --model mlp --steps 20 --warmup 5 > gpurun_out/r5h_mlp.log 2>&1 || { tail -20 gpurun_out/r5h_mlp.log; exit 1; }
  echo "$cfg $(tail -1 gpurun_out/r5h_mlp.log | cut -c1-260)"
done
tail -1 gpurun_out/r5h_mlp.log > gpurun_out/r5h_mlp.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r5h_prof_mlp" -o mlp --output-format csv -- python3 "$R/bench.py" \
  --model mlp --steps 40 --warmup 5 > "$R/gpurun_out/r5h_prof_mlp.log" 2>&1 || { echo "profile mlp failed"; exit 1; }
python3 "$R/scripts/graph_kernel_table.py" "$R/gpurun_out/r5h_prof_mlp/mlp_kernel_trace.csv" --title "mlp one-launch step r5h" --step-kernel k_mlp_train \
  > "$R/gpurun_out/r5h_mlp_graph_kernels.md" && head -12 "$R/gpurun_out/r5h_mlp_graph_kernels.md"
