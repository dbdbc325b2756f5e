#!/bin/bash
# Round-6 Y: world-2 rehearsal of the bench on one GPU (gloo control plane, xGMI IPC data plane) for every model
# the 8-GPU scaling run can take, after this round's comm / GEMM / BN changes.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
bash scripts/gpu_rehearse_world2.sh cnn hvd_cnn hvd_cnn_elastic mlp resnet50 resnet50_pp
