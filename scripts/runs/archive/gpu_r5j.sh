#!/bin/bash
# Round-5 J: one-launch MLP step v2 (sc1 hand-offs, counter barrier, overlapped backward loads)
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m pytest -x -v --timeout 120 --timeout-method thread tests/test_mlp_mega_gpu.py > gpurun_out/r5j_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|error|assert|passed|failed" gpurun_out/r5j_pytest.log | head -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/mlp_mega_phases.py > gpurun_out/r5j_phases.txt 2>&1 || { tail gpurun_out/r5j_phases.txt; exit 1; }
cat gpurun_out/r5j_phases.txt
for cfg in "PDE_MLP_MEGA=0" "PDE_MLP_MEGA=1"; do
  env $cfg timeout -k 10 200 python bench.py --model mlp --steps 20 --warmup 5 > gpurun_out/r5j_mlp.log 2>&1 || { tail -20 gpurun_out/r5j_mlp.log; exit 1; }
  echo "$cfg $(tail -1 gpurun_out/r5j_mlp.log | cut -c1-260)"
done
