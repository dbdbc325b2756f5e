#!/bin/bash
# Round-3 check M: folded Adam after the compute-copy fix: diagnostic, equivalence test, MLP sweep + trace.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 120 python scripts/diag_fold_opt.py > gpurun_out/r3m_diag.log 2>&1; cat gpurun_out/r3m_diag.log | tail -30
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -v --timeout 200 --timeout-method thread -k "folded or mlp" \
  > gpurun_out/r3m_pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed|^E " gpurun_out/r3m_pytest.log | tail -12
[ $rc -le 1 ] || exit $rc
MODELS="mlp" CONFIGS="PDE_MLP_FOLD_OPT=1;base" STEPS=50 REPS=2 bash scripts/gpu_envsweep.sh && cp gpurun_out/sweep.txt gpurun_out/r3m_sweep.txt
cd /tmp && PDE_MLP_FOLD_OPT=1 timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/tl_mlpfoldB" -o mlp --output-format csv \
    -- python3 "$R/bench.py" --model mlp --steps 40 --warmup 10 > "$R/gpurun_out/tl_mlpfoldB.log" 2>&1 || exit 1
cd "$R"; f=$(find gpurun_out/tl_mlpfoldB -name '*kernel_trace.csv' | head -1)
python3 scripts/graph_kernel_table.py "$f" --title "mlp, Adam folded into the backward launches" > gpurun_out/tl_mlpfoldB.md; head -16 gpurun_out/tl_mlpfoldB.md
