#!/bin/bash
# Round-3 check AE: CNN bench hipGraph kernel trace (k_cnn_train / k_cnn_reduce durations and gaps).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/tl_r3ae" -o cnn --output-format csv \
    -- python3 "$R/bench.py" --steps 60 --warmup 10 > "$R/gpurun_out/tl_r3ae.log" 2>&1 || exit 1
cd "$R"; f=$(find gpurun_out/tl_r3ae -name '*kernel_trace.csv' | head -1)
python3 scripts/timeline_gaps.py "$f" --last 200 --seq 12 > gpurun_out/r3ae_cnn_timeline.txt; cat gpurun_out/r3ae_cnn_timeline.txt
