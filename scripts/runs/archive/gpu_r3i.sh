#!/bin/bash
# Round-3 check I: world-2 rehearsal of the bench's multi-rank paths on one GPU (gloo between 2 ranks on
# cuda:0): the default CNN run WITH its secondary resnet50_pp child (PDE_BENCH_SECONDARY=force), mlp, resnet50,
# resnet50_pp with grouped units and with one micro-batch per unit.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out && export PYTHONUNBUFFERED=1 PDE_BACKEND=gloo
: > gpurun_out/r3i_w2.jsonl
run() {  # tag, env..., -- bench args
  local tag=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 "$@" > gpurun_out/w2_$tag.log 2>&1 || { tail -30 gpurun_out/w2_$tag.log; return 1; }
  grep '^{' gpurun_out/w2_$tag.log | tail -1 >> gpurun_out/r3i_w2.jsonl
  grep '^{' gpurun_out/w2_$tag.log | tail -1 | cut -c1-300
}
run cnn PDE_BENCH_SECONDARY=force -- --steps 10 --warmup 3 && \
run mlp X=1 -- --model mlp --steps 10 --warmup 3 && \
run resnet50 X=1 -- --model resnet50 --steps 10 --warmup 3 && \
run pp_grouped X=1 -- --model resnet50_pp --steps 10 --warmup 3 && \
run pp_g1 X=1 -- --model resnet50_pp --mb-group 1 --steps 10 --warmup 3
