#!/bin/bash
# Rehearse the bench's world > 1 path on the one-GPU box: 2 ranks on cuda:0 over gloo (PDE_BACKEND=gloo),
# per model.  RCCL itself needs one GPU per rank; this covers the DDP / fused-CNN data plane.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out && export PYTHONUNBUFFERED=1 PDE_BACKEND=gloo
for m in ${@:-cnn resnet50 mlp resnet50_pp}; do
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --model $m --steps 10 --warmup 3 > gpurun_out/w2_$m.log 2>&1 \
    || { tail -30 gpurun_out/w2_$m.log; exit 1; }
  grep '^{' gpurun_out/w2_$m.log | cut -c1-330
done
