#!/bin/bash
# Round-4 check H: BatchNorm fold with sharded statistics -- tests, A/B benches, kernel table; then the pipeline
# unit sweep (check G).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_bnfold_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r4h_pytest.log 2>&1 || { tail -30 gpurun_out/r4h_pytest.log; exit 1; }
tail -1 gpurun_out/r4h_pytest.log
: > gpurun_out/r4h_bench.jsonl
for m in "--model resnet50" "--model resnet50_stage --stage 1 --batch 8" "--model resnet50_stage --stage 2 --batch 8"; do
  for f in 1 0; do
    PDE_BN_FOLD=$f timeout -k 10 200 python bench.py $m --steps 30 --warmup 10 > gpurun_out/r4h_one.log 2>&1 || { tail -20 gpurun_out/r4h_one.log; exit 1; }
    tail -1 gpurun_out/r4h_one.log >> gpurun_out/r4h_bench.jsonl
    python -c "import json; d=json.loads(open('gpurun_out/r4h_one.log').read().strip().splitlines()[-1]); print('fold=$f', d['config']['model'], d['ms_per_step'], d['value'], json.dumps(d['config'].get('phases'))[:200])"
  done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/tl_r4h" -o rn --output-format csv \
    -- python3 "$R/bench.py" --model resnet50 --steps 30 --warmup 10 > "$R/gpurun_out/tl_r4h.log" 2>&1 || exit 1
cd "$R"; f=$(find gpurun_out/tl_r4h -name '*kernel_trace.csv' | head -1)
python3 scripts/graph_kernel_table.py "$f" --title "resnet50 r4h, BatchNorm folded (sharded statistics)" > gpurun_out/r4h_resnet50_graph_kernels.md; head -22 gpurun_out/r4h_resnet50_graph_kernels.md

