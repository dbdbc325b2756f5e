#!/bin/bash
# Round-4 check G: pipeline unit sweep for BASELINE configs 3/4 (VERDICT r3 ask 8): each stage at units of
# g x m8 micro-batches (grouped BatchNorm), g in {1, 2, 4}; scripts/pipeline_units.py turns the stage times into
# the predicted 2-GPU GPipe / 1F1B step per unit size.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
: > gpurun_out/r4g_stages.jsonl
for g in 1 2 4; do
  for st in 1 2; do
    timeout -k 10 200 python bench.py --model resnet50_stage --stage $st --batch $((8 * g)) --mb-group $g --steps 30 --warmup 10 \
      > gpurun_out/r4g_one.log 2>&1 || { tail -20 gpurun_out/r4g_one.log; exit 1; }
    tail -1 gpurun_out/r4g_one.log >> gpurun_out/r4g_stages.jsonl
    tail -1 gpurun_out/r4g_one.log | cut -c1-150
  done
done
python scripts/pipeline_units.py gpurun_out/r4g_stages.jsonl > gpurun_out/r4g_pipeline_units.md && cat gpurun_out/r4g_pipeline_units.md
