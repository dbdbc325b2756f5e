#!/bin/bash
# Round-5 X: split-K policy re-sweep after the first-write change (ring core) on ResNet-50 b32 and the m = 8 stages: per-block K-tile floor
# (PDE_GEMM_SPLIT_MIN_KT) x block target (PDE_GEMM_SPLIT_TARGET).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 PDE_BENCH_PHASES=0 PDE_BENCH_OVERHEADS=0
: > gpurun_out/r5x_sweep.txt
for kt in 16 8 4; do for tg in 256 512; do
  line="kt=$kt target=$tg"
  for m in "resnet50" "resnet50_stage --stage 1 --batch 8" "resnet50_stage --stage 2 --batch 8"; do
    PDE_GEMM_SPLIT_MIN_KT=$kt PDE_GEMM_SPLIT_TARGET=$tg timeout -k 10 200 python bench.py --model $m --steps 30 --warmup 10 \
      > gpurun_out/r5x_one.log 2>&1 || { tail -20 gpurun_out/r5x_one.log; exit 1; }
    line="$line $(tail -1 gpurun_out/r5x_one.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  done
  echo "$line" | tee -a gpurun_out/r5x_sweep.txt
done; done
