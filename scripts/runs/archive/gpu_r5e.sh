#!/bin/bash
# Round-5 E: the pipeline-unit stage table with the current kernels (stages 1/2 at g = 1, 2, 4 micro-batches of 8
# per unit), the 1-GPU whole-model rate, and kernel traces of the m = 8 stages (launch count / per-kernel time).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
: > gpurun_out/r5e_stages.jsonl
for g in 1 2 4; do for s in 1 2; do
  timeout -k 10 200 python bench.py --model resnet50_stage --stage $s --batch $((8 * g)) --mb-group $g --steps 30 --warmup 10 \
    > gpurun_out/r5e_one.log 2>&1 || { tail -20 gpurun_out/r5e_one.log; exit 1; }
  tail -1 gpurun_out/r5e_one.log >> gpurun_out/r5e_stages.jsonl
  echo "stage $s g $g $(tail -1 gpurun_out/r5e_one.log | cut -c150-230)"
done; done
timeout -k 10 200 python bench.py --model resnet50 --steps 30 --warmup 10 > gpurun_out/r5e_one.log 2>&1 || { tail -20 gpurun_out/r5e_one.log; exit 1; }
tail -1 gpurun_out/r5e_one.log > gpurun_out/r5e_resnet50.jsonl
python3 scripts/pipeline_units.py gpurun_out/r5e_stages.jsonl --one-gpu gpurun_out/r5e_resnet50.jsonl --json gpurun_out/r5e_pipeline_units.json \
  > gpurun_out/r5e_pipeline_units.md && cat gpurun_out/r5e_pipeline_units.md
cd /tmp && export TMPDIR=/tmp
for s in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r5e_prof_s$s" -o s$s --output-format csv -- python3 "$R/bench.py" \
    --model resnet50_stage --stage $s --batch 8 --steps 40 --warmup 5 > "$R/gpurun_out/r5e_prof_s$s.log" 2>&1 || { echo "profile s$s failed"; exit 1; }
  python3 "$R/scripts/graph_kernel_table.py" "$R/gpurun_out/r5e_prof_s$s/s${s}_kernel_trace.csv" --title "stage $s m8 r5e" --step-kernel k_optim \
    > "$R/gpurun_out/r5e_stage${s}_m8_graph_kernels.md" && head -14 "$R/gpurun_out/r5e_stage${s}_m8_graph_kernels.md"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r5e_prof_mlp" -o mlp --output-format csv -- python3 "$R/bench.py" \
  --model mlp --steps 40 --warmup 5 > "$R/gpurun_out/r5e_prof_mlp.log" 2>&1 || { echo "profile mlp failed"; exit 1; }
python3 "$R/scripts/graph_kernel_table.py" "$R/gpurun_out/r5e_prof_mlp/mlp_kernel_trace.csv" --title "mlp r5e" --step-kernel k_optim \
  > "$R/gpurun_out/r5e_mlp_graph_kernels.md" && head -14 "$R/gpurun_out/r5e_mlp_graph_kernels.md"
