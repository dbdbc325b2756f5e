#!/bin/bash
# Round-3 check E: BatchNorm (mask-from-x backward) + skinny-GEMM kernels, fused MLP, MLP bench skinny A/B,
# ResNet block backward with slab deferral on / off, PS ring test.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -v --timeout 200 \
  --timeout-method thread -k "batchnorm or skinny or linear or mlp" > gpurun_out/r3e_k.log 2>&1
rc=$?; echo "kernels rc=$rc"; grep -E "passed|failed|^E " gpurun_out/r3e_k.log | head -12
[ $rc -eq 0 ] || exit $rc
for sk in 1 0; do
  PDE_GEMM_SKINNY=$sk timeout -k 10 200 python bench.py --model mlp --steps 50 --warmup 10 > gpurun_out/r3e_mlp$sk.log 2>&1 || { tail -5 gpurun_out/r3e_mlp$sk.log; exit 1; }
  echo "skinny=$sk $(tail -1 gpurun_out/r3e_mlp$sk.log | cut -c1-260)"
done
for cfg in "PDE_OPTIM_NT=0" "PDE_OPTIM_BLOCKS=2048" "PDE_OPTIM_NT=0 PDE_OPTIM_BLOCKS=2048"; do
  env $cfg timeout -k 10 200 python bench.py --model mlp --steps 50 --warmup 10 > gpurun_out/r3e_mlpopt.log 2>&1 || { tail -5 gpurun_out/r3e_mlpopt.log; exit 1; }
  echo "[$cfg] $(tail -1 gpurun_out/r3e_mlpopt.log | cut -c1-200)"
done
for d in 1 0; do
  PDE_CONV_BN_DEFER=$d timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -x -q --timeout 200 \
    --timeout-method thread -k "resnet_blocks_backward" > gpurun_out/r3e_defer$d.log 2>&1
  rc=$?; echo "defer=$d rc=$rc"; grep -E "^E |passed|failed" gpurun_out/r3e_defer$d.log | head -12
  case $rc in 0|1) ;; *) exit $rc;; esac
done
timeout -k 10 300 python -u -m pytest tests/test_pipeline_gpu.py -v --timeout 200 --timeout-method thread \
  -k "parameter_server" > gpurun_out/r3e_ps.log 2>&1
echo "ps rc=$?"; grep -E "PASSED|FAILED|^E " gpurun_out/r3e_ps.log | head -12
