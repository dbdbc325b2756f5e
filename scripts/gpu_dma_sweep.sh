#!/bin/bash
# DMA GEMM core ring-depth sweep: numerics, ResNet-50 / MLP benches (ring vs dma auto), and per-shape GEMM
# tables (PDE_GEMM_LOG joined with a kernel trace) for forced 64x64 ring depths S and pair depths.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
PDE_GEMM_CORE=dma timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/dsw_pytest.log 2>&1
rc=$?; echo "dma pytest rc=$rc"; tail -3 gpurun_out/dsw_pytest.log
[ $rc -eq 0 ] || exit $rc
bench() {  # label, env...
  local label=$1; shift
  env "$@" timeout -k 10 200 python bench.py --model resnet50 --steps 30 --warmup 10 > gpurun_out/dsw_$label.log 2>&1 || { tail -5 gpurun_out/dsw_$label.log; return 1; }
  echo "$label $(tail -1 gpurun_out/dsw_$label.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
}
bench ring PDE_GEMM_CORE=ring || exit 1
bench dma_auto PDE_GEMM_CORE=dma || exit 1
bench dma64_auto PDE_GEMM_CORE=dma PDE_GEMM_DMA_TILE=64x64 || exit 1
for sv in 2 4 8; do bench dma64_s$sv PDE_GEMM_CORE=dma PDE_GEMM_DMA_TILE=64x64 PDE_DMA_S64=$sv || exit 1; done
for sp in 3 6; do bench dma64_p$sp PDE_GEMM_CORE=dma PDE_GEMM_DMA_TILE=64x64 PDE_DMA_SPAIR=$sp || exit 1; done
export TMPDIR=/tmp PDE_GEMM_LOG=1 PDE_BENCH_PHASES=0 PDE_BENCH_OVERHEADS=0
table() {  # label, env...
  local label=$1; shift
  cd /tmp && env "$@" timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/dsw_gs_$label" -o "r" --output-format csv \
    -- python3 "$R/bench.py" --no-graph --steps 3 --warmup 1 --model resnet50 > "$R/gpurun_out/dsw_gs_$label.log" 2>&1 || { echo "trace $label failed"; tail -5 "$R/gpurun_out/dsw_gs_$label.log"; cd "$R"; return 1; }
  cd "$R"
  f=$(find gpurun_out/dsw_gs_$label -name '*kernel_trace.csv' | head -1)
  python3 scripts/gemm_shape_table.py gpurun_out/dsw_gs_$label.log "$f" --steps 4 --title "resnet50 $label: GEMM launches of one eager step" > gpurun_out/dsw_gs_$label.md
  sed -n 3p gpurun_out/dsw_gs_$label.md
}
table dma_auto PDE_GEMM_CORE=dma || exit 1
for sv in 2 3 4 6 8; do table s$sv PDE_GEMM_CORE=dma PDE_GEMM_DMA_TILE=64x64 PDE_DMA_S64=$sv PDE_DMA_SPAIR=$([ $sv -ge 6 ] && echo 6 || echo 3) || exit 1; done
