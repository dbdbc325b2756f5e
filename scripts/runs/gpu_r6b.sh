#!/bin/bash
# Round-6 B: entry scripts on their default GPU paths (epoch hipGraphs): GPU tests + per-epoch images/s vs bench.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_entry_fast_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r6b_pytest.log 2>&1 || { tail -40 gpurun_out/r6b_pytest.log; exit 1; }
tail -6 gpurun_out/r6b_pytest.log
timeout -k 10 600 python scripts/entry_scripts_measure.py gpurun_out/r6_entry_scripts.jsonl > gpurun_out/r6b_entry.log 2>&1 || { tail -40 gpurun_out/r6b_entry.log; exit 1; }
cat gpurun_out/r6b_entry.log
