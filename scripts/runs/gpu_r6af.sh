#!/bin/bash
# Round-6 AF: grouped pipeline units (4 x m8) per stage after this round's changes.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for st in 1 2; do
  timeout -k 10 200 python bench.py --model resnet50_stage --stage $st --batch 32 --mb-group 4 --steps 40 --warmup 8 > gpurun_out/r6af_s$st.log 2>&1 || { tail -5 gpurun_out/r6af_s$st.log; exit 1; }
  grep '^{' gpurun_out/r6af_s$st.log | tail -1 | tee -a gpurun_out/r6af_units.jsonl | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])'
done
