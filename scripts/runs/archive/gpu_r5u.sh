#!/bin/bash
# Round-5 U: the pipeline-unit stage table re-measured after the first-write-stores change.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
: > gpurun_out/r5u_stages.jsonl
for g in 1 2 4; do for s in 1 2; do
  timeout -k 10 200 python bench.py --model resnet50_stage --stage $s --batch $((8 * g)) --mb-group $g --steps 30 --warmup 10 \
    > gpurun_out/r5u_one.log 2>&1 || { tail -20 gpurun_out/r5u_one.log; exit 1; }
  tail -1 gpurun_out/r5u_one.log >> gpurun_out/r5u_stages.jsonl
done; done
timeout -k 10 200 python bench.py --model resnet50 --steps 30 --warmup 10 > gpurun_out/r5u_one.log 2>&1 || { tail -20 gpurun_out/r5u_one.log; exit 1; }
tail -1 gpurun_out/r5u_one.log > gpurun_out/r5u_resnet50.jsonl
python3 scripts/pipeline_units.py gpurun_out/r5u_stages.jsonl --one-gpu gpurun_out/r5u_resnet50.jsonl --json gpurun_out/r5u_pipeline_units.json \
  > gpurun_out/r5u_pipeline_units.md && cat gpurun_out/r5u_pipeline_units.md
