#!/bin/bash
# Round-4 check I: cost attribution of the BatchNorm fold (PDE_BN_FOLD_DEBUG: 1 no finalize tail, 2 no statistics
# epilogue, 4 no A transform; timing only) + the fused-CNN kernel trace (train vs reduce kernel).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for cfg in "PDE_BN_FOLD=0" "PDE_BN_FOLD=1" "PDE_BN_FOLD_DEBUG=1" "PDE_BN_FOLD_DEBUG=3" "PDE_BN_FOLD_DEBUG=4" "PDE_BN_FOLD_DEBUG=7"; do
  env $cfg timeout -k 10 200 python bench.py --model resnet50 --steps 30 --warmup 10 > gpurun_out/r4i_one.log 2>&1 || { tail -20 gpurun_out/r4i_one.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4i_one.log').read().strip().splitlines()[-1]); p=d['config']['phases']['rank0_ms']; print('$cfg', d['ms_per_step'], 'fwd', p.get('fwd'), 'bwd', p.get('bwd'))"
done
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d "$R/gpurun_out/tl_r4i" -o cnn --output-format csv \
    -- python3 "$R/bench.py" --model cnn --steps 100 --warmup 20 > "$R/gpurun_out/tl_r4i.log" 2>&1 || exit 1
cd "$R"; f=$(find gpurun_out/tl_r4i -name '*kernel_trace.csv' | head -1)
python3 scripts/graph_kernel_table.py "$f" --title "cnn r4i" --step-kernel k_cnn_reduce > gpurun_out/r4i_cnn_graph_kernels.md; head -14 gpurun_out/r4i_cnn_graph_kernels.md
