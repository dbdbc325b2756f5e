#!/bin/bash
# Round-4 check D: BatchNorm folded into the convolutions -- correctness (fold vs unfolded, CPU reference,
# the existing ResNet block tests), then ResNet-50 / stage benches and the ResNet-50 graph kernel table.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_bnfold_gpu.py tests/test_models_gpu.py -k "bnfold or fold or resnet" -m gpu -v -x \
    --timeout 300 --timeout-method thread > gpurun_out/r4d_pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r4d_pytest.log | tail -14
[ $rc -eq 0 ] || { grep -E "^E " gpurun_out/r4d_pytest.log | head -30; exit $rc; }
: > gpurun_out/r4d_bench.jsonl
for m in "resnet50" "resnet50_stage --stage 1 --batch 8" "resnet50_stage --stage 2 --batch 8"; do
  timeout -k 10 200 python bench.py --model $m --steps 30 --warmup 10 > gpurun_out/r4d_one.log 2>&1 || { tail -20 gpurun_out/r4d_one.log; exit 1; }
  tail -1 gpurun_out/r4d_one.log >> gpurun_out/r4d_bench.jsonl
  tail -1 gpurun_out/r4d_one.log | cut -c1-160
  PDE_BN_FOLD=0 timeout -k 10 200 python bench.py --model $m --steps 30 --warmup 10 > gpurun_out/r4d_one.log 2>&1 || { tail -20 gpurun_out/r4d_one.log; exit 1; }
  tail -1 gpurun_out/r4d_one.log >> gpurun_out/r4d_bench.jsonl
  tail -1 gpurun_out/r4d_one.log | cut -c1-160
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/tl_r4d" -o rn --output-format csv \
    -- python3 "$R/bench.py" --model resnet50 --steps 30 --warmup 10 > "$R/gpurun_out/tl_r4d.log" 2>&1 || exit 1
cd "$R"; f=$(find gpurun_out/tl_r4d -name '*kernel_trace.csv' | head -1)
python3 scripts/graph_kernel_table.py "$f" --title "resnet50 r4d, BatchNorm folded into the convs" > gpurun_out/r4d_resnet50_graph_kernels.md; head -30 gpurun_out/r4d_resnet50_graph_kernels.md
