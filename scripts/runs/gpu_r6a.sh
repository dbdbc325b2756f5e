#!/bin/bash
# Round-6 A: GPU suite + smoke + driver-config bench after the advisor fixes (DDP stale views, MLP barrier wrap).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6a_pytest.log 2>&1 || { tail -30 gpurun_out/r6a_pytest.log; exit 1; }
tail -3 gpurun_out/r6a_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6a_smoke.log 2>&1 || { tail -20 gpurun_out/r6a_smoke.log; exit 1; }
cat gpurun_out/r6a_smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6a_bench.jsonl 2> gpurun_out/r6a_bench.err || { tail -20 gpurun_out/r6a_bench.err; exit 1; }
cut -c1-400 gpurun_out/r6a_bench.jsonl
