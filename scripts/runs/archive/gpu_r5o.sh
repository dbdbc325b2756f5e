#!/bin/bash
# Round-5 O: one-launch MLP final A/B (3 alternating runs each), phases, kernel trace.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mlp_mega_gpu.py > gpurun_out/r5o_pytest.log 2>&1 || { tail -30 gpurun_out/r5o_pytest.log; exit 1; }
tail -1 gpurun_out/r5o_pytest.log
timeout -k 10 120 python scripts/mlp_mega_phases.py > gpurun_out/r5o_phases.txt 2>&1 || { tail gpurun_out/r5o_phases.txt; exit 1; }
: > gpurun_out/r5o_mlp_ab.jsonl
for rep in 1 2 3; do for cfg in 0 1; do
  PDE_MLP_MEGA=$cfg timeout -k 10 200 python bench.py --model mlp --steps 20 --warmup 5 > gpurun_out/r5o_mlp.log 2>&1 || { tail -20 gpurun_out/r5o_mlp.log; exit 1; }
  tail -1 gpurun_out/r5o_mlp.log >> gpurun_out/r5o_mlp_ab.jsonl
  echo "mega=$cfg $(tail -1 gpurun_out/r5o_mlp.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r5o_prof_mlp" -o mlp --output-format csv -- python3 "$R/bench.py" \
  --model mlp --steps 40 --warmup 5 > "$R/gpurun_out/r5o_prof_mlp.log" 2>&1 || { echo "profile mlp failed"; exit 1; }
python3 "$R/scripts/graph_kernel_table.py" "$R/gpurun_out/r5o_prof_mlp/mlp_kernel_trace.csv" --title "mlp one-launch step r5o" --step-kernel k_mlp_train \
  > "$R/gpurun_out/r5o_mlp_graph_kernels.md" && head -12 "$R/gpurun_out/r5o_mlp_graph_kernels.md"
