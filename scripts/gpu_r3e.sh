#!/bin/bash
# Round-3 check E: isolate the ResNet block-backward failure (slab deferral on / off), PS ring test.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for d in 1 0; do
  PDE_CONV_BN_DEFER=$d timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -x -q --timeout 200 \
    --timeout-method thread -k "resnet_blocks_backward" > gpurun_out/r3e_defer$d.log 2>&1
  echo "defer=$d rc=$?"; grep -E "^E |passed|failed" gpurun_out/r3e_defer$d.log | head -12
done
timeout -k 10 300 python -u -m pytest tests/test_pipeline_gpu.py -v --timeout 200 --timeout-method thread \
  -k "parameter_server" > gpurun_out/r3e_ps.log 2>&1
echo "ps rc=$?"; grep -E "PASSED|FAILED|^E " gpurun_out/r3e_ps.log | head -12
