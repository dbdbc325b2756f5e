#!/bin/bash
# Round-4 check X: fused CNN store flavours 2 (all write-through) vs 3 (wide write-through, dword plain).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
: > gpurun_out/r4x_bench.txt
for rep in 1 2 3; do for cfg in "PDE_CNN_STORE=2" "PDE_CNN_STORE=3"; do
  env $cfg timeout -k 10 200 python bench.py --steps 300 --warmup 20 > gpurun_out/r4x_one.log 2>&1 || { tail -20 gpurun_out/r4x_one.log; exit 1; }
  tail -1 gpurun_out/r4x_one.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', d['ms_per_step'], d['value'])" | tee -a gpurun_out/r4x_bench.txt
done; done
: > gpurun_out/r4x_mlp.txt
for cfg in "PDE_OPTIM_NT=1" "PDE_OPTIM_NT=0" "PDE_OPTIM_NT=2" "PDE_OPTIM_BLOCKS=512" "PDE_OPTIM_BLOCKS=1224" "PDE_OPTIM_NT=1"; do
  env $cfg timeout -k 10 200 python bench.py --model mlp --steps 200 --warmup 20 > gpurun_out/r4x_one.log 2>&1 || { tail -20 gpurun_out/r4x_one.log; exit 1; }
  tail -1 gpurun_out/r4x_one.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', d['ms_per_step'], d['value'], d['config']['phases']['rank0_ms'])" | tee -a gpurun_out/r4x_mlp.txt
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r4x_prof_mlp" -o mlp --output-format csv -- python3 "$R/bench.py" --model mlp --steps 40 --warmup 5 > "$R/gpurun_out/r4x_prof_mlp.log" 2>&1 || { echo "profile failed"; tail -5 "$R/gpurun_out/r4x_prof_mlp.log"; exit 1; }
cd "$R" && python3 scripts/graph_kernel_table.py gpurun_out/r4x_prof_mlp/mlp_kernel_trace.csv --title "mlp r4x" > gpurun_out/r4x_mlp_graph_kernels.md 2>&1; head -25 gpurun_out/r4x_mlp_graph_kernels.md
