#!/bin/bash
# Round-4 check V: world-2 rehearsals on one GPU (ranks share the card: the one-launch BatchNorm is off there).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
bash scripts/gpu_rehearse_world2.sh resnet50 resnet50_pp hvd_cnn cnn mlp
