#!/bin/bash
# Round-5 checks: new GPU tests (xGMI failure words, side-stream BatchNorm mix, elastic detection, Horovod-elastic
# kill), DMA core (pipelined) vs ring on ResNet-50, CNN bench attribution, hvd_cnn_elastic bench.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -m pytest -x -v --timeout 300 --timeout-method thread tests/test_xgmi_fail_gpu.py \
  tests/test_elastic_gpu.py > gpurun_out/r5d_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/r5d_pytest.log | tail -12
case $rc in 0|1) ;; *) exit $rc ;; esac  # a failed assertion is no GPU fault: go on to the benches
PDE_GEMM_CORE=dma timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/r5d_dma_pytest.log 2>&1 || { tail -20 gpurun_out/r5d_dma_pytest.log; exit 1; }
echo "dma numerics ok"
bench() {  # label, model, env...
  local label=$1 model=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --model $model --steps 30 --warmup 10 > gpurun_out/r5d_$label.log 2>&1 || { tail -5 gpurun_out/r5d_$label.log; return 1; }
  echo "$label $(tail -1 gpurun_out/r5d_$label.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
}
bench ring resnet50 PDE_GEMM_CORE=ring || exit 1
bench dma resnet50 PDE_GEMM_CORE=dma || exit 1
for sv in 2 3 4; do bench dma64_s$sv resnet50 PDE_GEMM_CORE=dma PDE_GEMM_DMA_TILE=64x64 PDE_DMA_S64=$sv PDE_DMA_SPAIR=3 || exit 1; done
bench dma128x64 resnet50 PDE_GEMM_CORE=dma PDE_GEMM_DMA_TILE=128x64 || exit 1
bench mlp_ring mlp PDE_GEMM_CORE=ring || exit 1
bench mlp_dma mlp PDE_GEMM_CORE=dma || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r5d_cnn_driver.log 2>&1 || { tail -5 gpurun_out/r5d_cnn_driver.log; exit 1; }
tail -1 gpurun_out/r5d_cnn_driver.log
bench hvd_elastic hvd_cnn_elastic || exit 1
export TMPDIR=/tmp PDE_GEMM_LOG=1 PDE_BENCH_PHASES=0 PDE_BENCH_OVERHEADS=0
cd /tmp && PDE_GEMM_CORE=dma timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r5d_gs_dma" -o "r" --output-format csv \
  -- python3 "$R/bench.py" --no-graph --steps 3 --warmup 1 --model resnet50 > "$R/gpurun_out/r5d_gs_dma.log" 2>&1 || { echo "trace failed"; exit 1; }
cd "$R"
f=$(find gpurun_out/r5d_gs_dma -name '*kernel_trace.csv' | head -1)
python3 scripts/gemm_shape_table.py gpurun_out/r5d_gs_dma.log "$f" --steps 4 --title "resnet50 dma (pipelined): GEMM launches of one eager step" > gpurun_out/r5d_gs_dma.md
sed -n 3p gpurun_out/r5d_gs_dma.md
