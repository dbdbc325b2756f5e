#!/bin/bash
# Round-5 ZE: the fused MLP update's w / m / v loaded at the end of the previous window (PDE_MLP_EARLY) --
# numerics, phase stamps, alternating A/B.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mlp_mega_gpu.py \
  > gpurun_out/r5ze_pytest.log 2>&1 || { tail -30 gpurun_out/r5ze_pytest.log; exit 1; }
tail -1 gpurun_out/r5ze_pytest.log
timeout -k 10 120 python scripts/mlp_mega_phases.py > gpurun_out/r5ze_phases.txt 2>&1 || { tail -20 gpurun_out/r5ze_phases.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r5ze_phases.txt | tail -24
: > gpurun_out/r5ze_mlp_ab.jsonl
for rep in 1 2 3; do for e in 1 0; do
  PDE_MLP_EARLY=$e timeout -k 10 200 python bench.py --model mlp --steps 200 --warmup 20 > gpurun_out/r5ze_one.log 2>&1 || { tail -20 gpurun_out/r5ze_one.log; exit 1; }
  echo "{\"early\": $e, \"rec\": $(tail -1 gpurun_out/r5ze_one.log)}" >> gpurun_out/r5ze_mlp_ab.jsonl
  echo "early=$e $(tail -1 gpurun_out/r5ze_one.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done; done
