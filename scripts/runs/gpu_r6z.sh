#!/bin/bash
# Round-6 Z: split-K policy sweep at the pipeline micro-batch (stage 1 / 2, m = 8) after this round's GEMM / BN changes.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
bench() {  # label, args...
  local label=$1; shift
  timeout -k 10 200 python bench.py "$@" > gpurun_out/r6z_$label.log 2>&1 || { tail -5 gpurun_out/r6z_$label.log; return 1; }
  echo "$label $(grep '^{' gpurun_out/r6z_$label.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
}
for st in 2 1; do
  S="--model resnet50_stage --stage $st --batch 8 --steps 40 --warmup 5"
  bench s${st}_base $S || exit 1
  PDE_GEMM_SPLIT_MIN_KT=4 bench s${st}_kt4 $S || exit 1
  PDE_GEMM_PAIR_BALANCE=1 bench s${st}_bal $S || exit 1
  PDE_GEMM_SPLIT_TARGET=512 bench s${st}_t512 $S || exit 1
  PDE_GEMM_SPLIT_TARGET=512 PDE_GEMM_SPLIT_MIN_KT=4 bench s${st}_t512kt4 $S || exit 1
  PDE_GEMM_SPLIT_TARGET=128 bench s${st}_t128 $S || exit 1
  bench s${st}_base2 $S || exit 1
done
