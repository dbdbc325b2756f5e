#!/bin/bash
# Round-3 check N: fused CNN with paired-pixel conv1 gathers (x / shifted-copy x1): CNN tests, phase stamps,
# bench x3; then a world-4 rehearsal (4 ranks on one GPU, gloo) of resnet50_pp = pp2 x dp2 (the DDP-over-stage
# path of config 4).
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py tests/test_xgmi_gpu.py -v --timeout 120 --timeout-method thread \
  -k "cnn or dropout" > gpurun_out/r3n_pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed|^E " gpurun_out/r3n_pytest.log | tail -20
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python scripts/cnn_phase_stamps.py > gpurun_out/r3n_stamps.log 2>&1; tail -16 gpurun_out/r3n_stamps.log
MODELS="cnn" CONFIGS="base" REPS=3 STEPS=50 bash scripts/gpu_envsweep.sh && cp gpurun_out/sweep.txt gpurun_out/r3n_sweep_cnn.txt
PDE_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port 29541 bench.py --gpus 4 --model resnet50_pp --steps 5 --warmup 2 > gpurun_out/w4_pp.log 2>&1 \
  || { tail -30 gpurun_out/w4_pp.log; exit 1; }
grep '^{' gpurun_out/w4_pp.log | tail -1 | cut -c1-400
