#!/bin/bash
# Round-5 ZJ: the headline at the driver's own configuration (bench.py --gpus 1 --steps 20 --warmup 5), three runs.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
: > gpurun_out/r5zj_driver_config.jsonl
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5zj_one.log 2>&1 || { tail -20 gpurun_out/r5zj_one.log; exit 1; }
  grep '^{' gpurun_out/r5zj_one.log | tail -1 >> gpurun_out/r5zj_driver_config.jsonl
  tail -1 gpurun_out/r5zj_driver_config.jsonl | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["steps"], d["warmup"], d["ms_per_step"], d["value"])'
done
