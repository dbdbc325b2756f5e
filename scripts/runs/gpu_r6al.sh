#!/bin/bash
# Round-6 AL: one-launch BatchNorm grid knobs re-swept on the end-of-round code (ResNet-50 b32, stage 1 m8).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
bench() {  # label, args...
  local label=$1; shift
  timeout -k 10 200 python bench.py "$@" > gpurun_out/r6al_$label.log 2>&1 || { tail -5 gpurun_out/r6al_$label.log; return 1; }
  echo "$label $(grep '^{' gpurun_out/r6al_$label.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
}
R50="--model resnet50 --steps 30 --warmup 10"
bench r50_base $R50 || exit 1
PDE_BN_CHUNKS=64 bench r50_c64 $R50 || exit 1
PDE_BN_CHUNKS=256 bench r50_c256 $R50 || exit 1
PDE_BN_BLOCKS=128 bench r50_b128 $R50 || exit 1
PDE_BN_RC8=0 bench r50_norc8 $R50 || exit 1
PDE_BN_RC16=1 bench r50_rc16 $R50 || exit 1
bench r50_base2 $R50 || exit 1
S1="--model resnet50_stage --stage 1 --batch 8 --steps 40 --warmup 5"
bench s1_base $S1 || exit 1
PDE_BN_CHUNKS=64 bench s1_c64 $S1 || exit 1
PDE_BN_BLOCKS=128 bench s1_b128 $S1 || exit 1
