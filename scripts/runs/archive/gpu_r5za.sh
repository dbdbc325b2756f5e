#!/bin/bash
# Round-5 ZA: MLP weight tiles updated straight from their gradient accumulators (PDE_MLP_FUSE) and BatchNorm
# write-through by default -- numerics, MLP phase stamps, alternating MLP A/B, ResNet-50 / stage benches.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mlp_mega_gpu.py tests/test_kernels_gpu.py \
  > gpurun_out/r5za_pytest.log 2>&1 || { tail -30 gpurun_out/r5za_pytest.log; exit 1; }
tail -1 gpurun_out/r5za_pytest.log
timeout -k 10 120 python scripts/mlp_mega_phases.py > gpurun_out/r5za_phases.txt 2>&1 || { tail -20 gpurun_out/r5za_phases.txt; exit 1; }
PDE_MLP_FUSE=0 timeout -k 10 120 python scripts/mlp_mega_phases.py > gpurun_out/r5za_phases_unfused.txt 2>&1 || { tail -20 gpurun_out/r5za_phases_unfused.txt; exit 1; }
tail -3 gpurun_out/r5za_phases.txt gpurun_out/r5za_phases_unfused.txt
: > gpurun_out/r5za_mlp_ab.jsonl
for rep in 1 2 3; do for f in 1 0; do
  PDE_MLP_FUSE=$f timeout -k 10 200 python bench.py --model mlp --steps 200 --warmup 20 > gpurun_out/r5za_one.log 2>&1 || { tail -20 gpurun_out/r5za_one.log; exit 1; }
  echo "{\"fuse\": $f, \"rec\": $(tail -1 gpurun_out/r5za_one.log)}" >> gpurun_out/r5za_mlp_ab.jsonl
  echo "fuse=$f $(tail -1 gpurun_out/r5za_one.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done; done
: > gpurun_out/r5za_resnet.jsonl
for m in "resnet50" "resnet50_stage --stage 1 --batch 32 --mb-group 4" "resnet50_stage --stage 2 --batch 32 --mb-group 4"; do
  timeout -k 10 200 python bench.py --model $m --steps 30 --warmup 10 > gpurun_out/r5za_one.log 2>&1 || { tail -20 gpurun_out/r5za_one.log; exit 1; }
  tail -1 gpurun_out/r5za_one.log >> gpurun_out/r5za_resnet.jsonl
  echo "$m $(tail -1 gpurun_out/r5za_one.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done
