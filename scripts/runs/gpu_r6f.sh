#!/bin/bash
# Round-6 F: pp2 x dp2 on one GPU -- does a small two-shot grid avoid starving the other pipeline's kernels?
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for blocks in 8 1; do
  PDE_XGMI2_BLOCKS=$blocks PDE_BACKEND=gloo PDE_P2P_TIMEOUT_S=10 PDE_XGMI_TIMEOUT_S=10 timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 --master-addr 127.0.0.1 --master-port 2961$blocks scripts/diag_pipe_dp.py 1f1b graph > gpurun_out/r6f_diag_b$blocks.log 2>&1
  echo "blocks=$blocks diag rc=$?"
  grep "^\[ " gpurun_out/r6f_diag_b$blocks.log | head -30
done
