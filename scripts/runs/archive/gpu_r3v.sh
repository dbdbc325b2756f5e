#!/bin/bash
# Round-3 check V: fused CNN with the reduction inside k_cnn_train (grid barrier, PDE_CNN_FUSED_TAIL): CNN tests,
# bench with the tail on (bench default at world 1) / off, hipGraph kernel trace.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py tests/test_xgmi_gpu.py -v --timeout 120 --timeout-method thread \
  -k "cnn or dropout" > gpurun_out/r3v_pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed|^E " gpurun_out/r3v_pytest.log | tail -16
[ $rc -eq 0 ] || exit 1
MODELS="cnn" CONFIGS="base;PDE_CNN_FUSED_TAIL=0" REPS=3 STEPS=100 bash scripts/gpu_envsweep.sh && cp gpurun_out/sweep.txt gpurun_out/r3v_sweep.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/tl_cnntail" -o cnn --output-format csv \
    -- python3 "$R/bench.py" --steps 60 --warmup 10 > "$R/gpurun_out/tl_cnntail.log" 2>&1 || exit 1
cd "$R"; f=$(find gpurun_out/tl_cnntail -name '*kernel_trace.csv' | head -1)
python3 scripts/graph_kernel_table.py "$f" --title "cnn, single-launch step (fused tail)" > gpurun_out/tl_cnntail.md; head -12 gpurun_out/tl_cnntail.md
