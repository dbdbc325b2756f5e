#!/bin/bash
# GEMM engine change check: kernel + model GPU tests, then the MLP and ResNet-50 benches.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gemm_tests.log 2>&1
rc=$?; tail -4 gpurun_out/gemm_tests.log; [ $rc -eq 0 ] || { grep -E "^E |Error" gpurun_out/gemm_tests.log | head -30; exit $rc; }
for m in mlp resnet50; do
  timeout -k 10 300 python bench.py --model $m --steps 30 --warmup 10 > gpurun_out/chk_${m}.log 2>&1 || { tail -5 gpurun_out/chk_${m}.log; exit 1; }
  echo "$m: $(tail -1 gpurun_out/chk_${m}.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], "img/s", r["ms_per_step"], "ms/step")')"
done
