#!/bin/bash
# Round-6 P: streamed low-K GEMM (K <= 128): numerics, ResNet-50 / stage-1 A/B, grid-cap sweep, shape table.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6p_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r6p_pytest.log
[ $rc -eq 0 ] || exit $rc
bench() {  # label, args...
  local label=$1; shift
  timeout -k 10 200 python bench.py "$@" > gpurun_out/r6p_$label.log 2>&1 || { tail -5 gpurun_out/r6p_$label.log; return 1; }
  echo "$label $(grep '^{' gpurun_out/r6p_$label.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
}
bench resnet50 --model resnet50 --steps 30 --warmup 10 || exit 1
PDE_GEMM_LOWK=0 bench resnet50_off --model resnet50 --steps 30 --warmup 10 || exit 1
PDE_GEMM_LOWK_BLOCKS=256 bench resnet50_b256 --model resnet50 --steps 30 --warmup 10 || exit 1
PDE_GEMM_LOWK_BLOCKS=1024 bench resnet50_b1024 --model resnet50 --steps 30 --warmup 10 || exit 1
bench stage1 --model resnet50_stage --stage 1 --batch 8 --steps 40 --warmup 5 || exit 1
PDE_GEMM_LOWK=0 bench stage1_off --model resnet50_stage --stage 1 --batch 8 --steps 40 --warmup 5 || exit 1
export TMPDIR=/tmp PDE_GEMM_LOG=1 PDE_BENCH_PHASES=0 PDE_BENCH_OVERHEADS=0
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r6p_gs" -o "r" --output-format csv \
  -- python3 "$R/bench.py" --no-graph --steps 3 --warmup 1 --model resnet50 > "$R/gpurun_out/r6p_gs.log" 2>&1 || { echo "trace failed"; exit 1; }
cd "$R"
f=$(find gpurun_out/r6p_gs -name '*kernel_trace.csv' | head -1)
python3 scripts/gemm_shape_table.py gpurun_out/r6p_gs.log "$f" --steps 4 --title "resnet50 b32: GEMM launches of one eager step (low-K path on)" > gpurun_out/r6p_gemm_shapes.md
sed -n 1,4p gpurun_out/r6p_gemm_shapes.md; grep lowk gpurun_out/r6p_gemm_shapes.md
