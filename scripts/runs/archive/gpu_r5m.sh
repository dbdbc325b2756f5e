#!/bin/bash
# Round-5 M: BatchNorm single-chunk fast path (numerics + A/B), one-launch MLP (gpu_r5j), Horovod world-2 graph
# mode engine counters, and the ring GEMM compiled for 3 waves / SIMD (no spills in the 64x64 tiles) A/B.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "batchnorm" \
  tests/test_bn_sidestream_gpu.py tests/test_models_gpu.py > gpurun_out/r5m_bn_pytest.log 2>&1
rc=$?; echo "bn pytest rc=$rc"; tail -3 gpurun_out/r5m_bn_pytest.log
[ $rc -eq 0 ] || exit $rc
bench() {  # label, model args..., env via BENV
  local label=$1; shift
  env $BENV timeout -k 10 200 python bench.py --model "$@" --steps 30 --warmup 10 > gpurun_out/r5m_$label.log 2>&1 || { tail -5 gpurun_out/r5m_$label.log; return 1; }
  echo "$label $(tail -1 gpurun_out/r5m_$label.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  tail -1 gpurun_out/r5m_$label.log >> gpurun_out/r5m_bench.jsonl
}
: > gpurun_out/r5m_bench.jsonl
for rows in 1024 0 512 2048; do
  BENV="PDE_BN_SINGLE_ROWS=$rows" bench r50_bn$rows resnet50 || exit 1
  BENV="PDE_BN_SINGLE_ROWS=$rows" bench s1_bn$rows resnet50_stage --stage 1 --batch 8 || exit 1
  BENV="PDE_BN_SINGLE_ROWS=$rows" bench s2_bn$rows resnet50_stage --stage 2 --batch 8 || exit 1
done
bash scripts/runs/archive/gpu_r5l.sh || exit 1
# the 3-waves/SIMD ring GEMM (built before the BatchNorm change: compare with PDE_BN_SINGLE_ROWS=0)
cp pytorch_distributed_examples_amd/_C.cpython-310-x86_64-linux-gnu.so /tmp/_C_default.so
cp variants/_C_wpe3.so pytorch_distributed_examples_amd/_C.cpython-310-x86_64-linux-gnu.so
BENV="PDE_BN_SINGLE_ROWS=0" bench r50_wpe3 resnet50
BENV="PDE_BN_SINGLE_ROWS=0" bench s2_wpe3 resnet50_stage --stage 2 --batch 8
BENV="PDE_BN_SINGLE_ROWS=0" bench mlp_wpe3 mlp
cp /tmp/_C_default.so pytorch_distributed_examples_amd/_C.cpython-310-x86_64-linux-gnu.so
BENV="PDE_BN_SINGLE_ROWS=0" bench r50_wpe4 resnet50
