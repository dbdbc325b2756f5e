#!/bin/bash
# LDS-DMA GEMM core: numerics under PDE_GEMM_CORE=dma, ResNet-50 / MLP benches ring vs dma, GEMM shape tables.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
PDE_GEMM_CORE=dma timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py tests/test_bnfold_gpu.py -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/dma_pytest.log 2>&1
rc=$?; echo "dma pytest rc=$rc"; tail -15 gpurun_out/dma_pytest.log
[ $rc -eq 0 ] || exit $rc
for core in ring dma; do
  for m in resnet50 mlp; do
    PDE_GEMM_CORE=$core timeout -k 10 200 python bench.py --model $m --steps 30 --warmup 10 > gpurun_out/dma_bench_${core}_$m.log 2>&1 || { tail -5 gpurun_out/dma_bench_${core}_$m.log; exit 1; }
    echo "$core $m $(tail -1 gpurun_out/dma_bench_${core}_$m.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
for t in default 64x64 128x64 128x128; do
  if [ $t = default ]; then unset PDE_GEMM_DMA_TILE; else export PDE_GEMM_DMA_TILE=$t; fi
  PDE_GEMM_CORE=dma timeout -k 10 200 python bench.py --model resnet50 --steps 30 --warmup 10 > gpurun_out/dma_tile_$t.log 2>&1 || { tail -5 gpurun_out/dma_tile_$t.log; exit 1; }
  echo "tile $t $(tail -1 gpurun_out/dma_tile_$t.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done
unset PDE_GEMM_DMA_TILE
export TMPDIR=/tmp PDE_GEMM_LOG=1 PDE_BENCH_PHASES=0
for core in ring dma; do
  cd /tmp && PDE_GEMM_CORE=$core timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/gsd_$core" -o "r" --output-format csv \
    -- python3 "$R/bench.py" --no-graph --steps 3 --warmup 1 --model resnet50 > "$R/gpurun_out/gsd_$core.log" 2>&1 || { echo "trace failed"; tail -5 "$R/gpurun_out/gsd_$core.log"; exit 1; }
  cd "$R"
  f=$(find gpurun_out/gsd_$core -name '*kernel_trace.csv' | head -1)
  python3 scripts/gemm_shape_table.py gpurun_out/gsd_$core.log "$f" --steps 4 --title "resnet50 $core core: GEMM launches of one eager step" > gpurun_out/gsd_$core.md
  head -4 gpurun_out/gsd_$core.md
done
