#!/bin/bash
# Round-5 S: BatchNorm launch-shape knobs re-swept with the current kernels (ResNet-50 b32 and stage 2 at m = 8).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 PDE_BENCH_PHASES=0 PDE_BENCH_OVERHEADS=0
: > gpurun_out/r5s_sweep.txt
for cfg in "BASE=1" "PDE_BN_CHUNKS=64" "PDE_BN_CHUNKS=256" "PDE_BN_BLOCKS=128" "PDE_BN_BLOCKS=512" "PDE_BN_RC16=1" "PDE_BN_WT=1" "PDE_BN_RC8=0" "BASE=2"; do
  line="$cfg"
  for m in "resnet50" "resnet50_stage --stage 2 --batch 8" "resnet50_stage --stage 1 --batch 32 --mb-group 4"; do
    env $cfg timeout -k 10 200 python bench.py --model $m --steps 30 --warmup 10 > gpurun_out/r5s_one.log 2>&1 || { tail -20 gpurun_out/r5s_one.log; exit 1; }
    line="$line $(tail -1 gpurun_out/r5s_one.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  done
  echo "$line" | tee -a gpurun_out/r5s_sweep.txt
done
