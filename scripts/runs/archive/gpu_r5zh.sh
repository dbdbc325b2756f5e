#!/bin/bash
# Round-5 ZH: fused MLP window loads issued BEFORE the barrier's arrive (drain and load latency overlap) --
# numerics, sub-phase clocks, alternating bench against the early-state-off and unfused forms.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mlp_mega_gpu.py \
  > gpurun_out/r5zh_pytest.log 2>&1 || { tail -30 gpurun_out/r5zh_pytest.log; exit 1; }
tail -1 gpurun_out/r5zh_pytest.log
timeout -k 10 120 python scripts/mlp_mega_phases.py > gpurun_out/r5zh_phases.txt 2>&1 || { tail -20 gpurun_out/r5zh_phases.txt; exit 1; }
grep -E "^B|sum" gpurun_out/r5zh_phases.txt | tail -26
: > gpurun_out/r5zh_mlp_ab.jsonl
for rep in 1 2 3; do for cfg in "X=1" "PDE_MLP_EARLY=0" "PDE_MLP_FUSE=0"; do
  env $cfg timeout -k 10 200 python bench.py --model mlp --steps 200 --warmup 20 > gpurun_out/r5zh_one.log 2>&1 || { tail -20 gpurun_out/r5zh_one.log; exit 1; }
  echo "{\"cfg\": \"$cfg\", \"rec\": $(tail -1 gpurun_out/r5zh_one.log)}" >> gpurun_out/r5zh_mlp_ab.jsonl
  echo "$cfg $(tail -1 gpurun_out/r5zh_one.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done; done
