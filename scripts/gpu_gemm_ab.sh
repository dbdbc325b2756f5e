#!/bin/bash
# GEMM engine change check: kernel/model tests, then the MLP and ResNet-50 benches with the new path and
# with the A/B switch (PDE_GEMM_INKERNEL_SPLITK=1: split-K combined in-kernel by the last K-slice).
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/gemm_tests.log 2>&1
rc=$?; tail -4 gpurun_out/gemm_tests.log; [ $rc -le 1 ] || exit $rc
for m in mlp resnet50; do
  for ab in 0 1; do
    if [ $ab = 1 ]; then export PDE_GEMM_INKERNEL_SPLITK=1; else unset PDE_GEMM_INKERNEL_SPLITK; fi
    timeout -k 10 300 python bench.py --model $m --steps 30 --warmup 10 > gpurun_out/ab_${m}_$ab.log 2>&1 || { tail -5 gpurun_out/ab_${m}_$ab.log; exit 1; }
    echo "$m inkernel_splitk=$ab: $(tail -1 gpurun_out/ab_${m}_$ab.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], "img/s", r["ms_per_step"], "ms/step")')"
  done
done
