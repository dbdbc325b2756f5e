#!/bin/bash
# Round-5 L: one-launch MLP (tests, phases, bench A/B) + the Horovod engine's world-2 graph-mode rehearsal
# (two ranks sharing the card over gloo + the xGMI data plane: bit_allreduces must stay ~flat in graph mode).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
bash scripts/runs/archive/gpu_r5j.sh || exit $?
PDE_BACKEND=gloo timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29541 bench.py --gpus 2 --model hvd_cnn --steps 20 --warmup 5 > gpurun_out/r5l_hvd_w2.log 2>&1 \
  || { tail -30 gpurun_out/r5l_hvd_w2.log; exit 1; }
grep '^{' gpurun_out/r5l_hvd_w2.log > gpurun_out/r5l_hvd_w2.jsonl
python -c "
import json
d = json.loads(open('gpurun_out/r5l_hvd_w2.jsonl').read().splitlines()[-1])
print('hvd w2', d['ms_per_step'], d['config'].get('hipgraph'), d['config'].get('engine'))
"
