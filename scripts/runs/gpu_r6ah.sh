#!/bin/bash
# Round-6 AH: store-mode knobs re-checked at the pipeline micro-batch (stage 2, m = 8) and ResNet-50 b32.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
bench() {  # label, args...
  local label=$1; shift
  timeout -k 10 200 python bench.py "$@" > gpurun_out/r6ah_$label.log 2>&1 || { tail -5 gpurun_out/r6ah_$label.log; return 1; }
  echo "$label $(grep '^{' gpurun_out/r6ah_$label.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
}
S2="--model resnet50_stage --stage 2 --batch 8 --steps 40 --warmup 5"
bench s2_base $S2 || exit 1
PDE_OPTIM_NT=1 bench s2_nt1 $S2 || exit 1
PDE_OPTIM_NT=2 bench s2_nt2 $S2 || exit 1
PDE_BN_WT=0 bench s2_bnwt0 $S2 || exit 1
PDE_GEMM_WT=0 bench s2_gemmwt0 $S2 || exit 1
bench s2_base2 $S2 || exit 1
R50="--model resnet50 --steps 30 --warmup 10"
bench r50_base $R50 || exit 1
PDE_OPTIM_NT=2 bench r50_nt2 $R50 || exit 1
PDE_BN_WT=0 bench r50_bnwt0 $R50 || exit 1
bench r50_base2 $R50 || exit 1
