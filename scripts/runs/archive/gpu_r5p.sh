#!/bin/bash
# Round-5 P: full GPU suite + smoke + default bench + world-2 rehearsals (resnet50_pp record fields, mlp, cnn).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r5p_pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5p_pytest.log | tail -12
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5p_smoke.log 2>&1 || { tail -20 gpurun_out/r5p_smoke.log; exit 1; }
tail -1 gpurun_out/r5p_smoke.log
timeout -k 10 200 python bench.py > gpurun_out/r5p_default.log 2>&1 && tail -1 gpurun_out/r5p_default.log | cut -c1-300
bash scripts/gpu_rehearse_world2.sh resnet50_pp mlp cnn > gpurun_out/r5p_world2.txt 2>&1; echo "w2 rc=$?"; cut -c1-400 gpurun_out/r5p_world2.txt
