#!/bin/bash
# Round-5 Z: write-through BatchNorm outputs (PDE_BN_WT=1) A/B, alternating runs.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 PDE_BENCH_PHASES=0 PDE_BENCH_OVERHEADS=0
: > gpurun_out/r5z_ab.txt
for rep in 1 2 3; do for wt in 0 1; do
  line="wt=$wt"
  for m in "resnet50" "resnet50_stage --stage 1 --batch 32 --mb-group 4" "resnet50_stage --stage 2 --batch 32 --mb-group 4" "resnet50_stage --stage 2 --batch 8"; do
    PDE_BN_WT=$wt timeout -k 10 200 python bench.py --model $m --steps 30 --warmup 10 > gpurun_out/r5z_one.log 2>&1 || { tail -20 gpurun_out/r5z_one.log; exit 1; }
    line="$line $(tail -1 gpurun_out/r5z_one.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  done
  echo "$line" | tee -a gpurun_out/r5z_ab.txt
done; done
