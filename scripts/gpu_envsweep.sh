#!/bin/bash
# Environment-switch sweep: for each model in MODELS, bench.py under each config of CONFIGS (";"-separated
# lists of VAR=value assignments, "base" = no change).  One JSON summary line per run -> gpurun_out/sweep.txt.
#   MODELS="resnet50 mlp" CONFIGS="base;PDE_BN_CHUNKS=256;PDE_OPTIM_NT=0" bash scripts/gpu_envsweep.sh
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
: > gpurun_out/sweep.txt
IFS=';' read -ra CFGS <<< "${CONFIGS:-base}"
for m in ${MODELS:-resnet50}; do
  for rep in $(seq 1 ${REPS:-1}); do
    for c in "${CFGS[@]}"; do
      envs=(); [ "$c" = "base" ] || read -ra envs <<< "$c"
      env "${envs[@]}" timeout -k 10 200 python bench.py --model $m --steps ${STEPS:-30} --warmup 10 ${BENCH_ARGS:-} \
        > gpurun_out/sweep_one.log 2>&1 || { tail -8 gpurun_out/sweep_one.log; exit 1; }
      line="$m [$c] $(tail -1 gpurun_out/sweep_one.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], "img/s", r["ms_per_step"], "ms/step")')"
      echo "$line" | tee -a gpurun_out/sweep.txt
    done
  done
done
