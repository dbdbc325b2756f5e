#!/bin/bash
# Round-3 check F: pipeline stage benches at micro-batch 4 / 8 / 32 (stage 2 was crashing in hipGraph capture:
# its static input is now a leaf), then the hipGraph kernel tables of mlp / resnet50 / both stages at m=8.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 PYTHONFAULTHANDLER=1
: > gpurun_out/r3f_bench.jsonl
for m in "resnet50_stage --stage 2 --batch 8" "resnet50_stage --stage 1 --batch 8" \
         "resnet50_stage --stage 1 --batch 4" "resnet50_stage --stage 2 --batch 4" \
         "resnet50_stage --stage 1 --batch 32" "resnet50_stage --stage 2 --batch 32"; do
  timeout -k 10 200 python bench.py --model $m --steps 30 --warmup 10 > gpurun_out/r3f_one.log 2>&1 || { tail -30 gpurun_out/r3f_one.log; exit 1; }
  tail -1 gpurun_out/r3f_one.log >> gpurun_out/r3f_bench.jsonl
  tail -1 gpurun_out/r3f_one.log | cut -c1-200
done
bash scripts/runs/archive/gpu_r3c.sh
