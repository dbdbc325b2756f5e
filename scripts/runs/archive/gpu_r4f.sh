#!/bin/bash
# Round-4 check F: BatchNorm fold (arrival moved to the block end) and the GEMM register budget (waves per EU 4
# vs 2: the 64x64 FAST tiles spill ~32 VGPRs at the 128-VGPR cap) -- ResNet-50 and stage benches, A/B.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_bnfold_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r4f_pytest.log 2>&1 || { tail -30 gpurun_out/r4f_pytest.log; exit 1; }
tail -1 gpurun_out/r4f_pytest.log
: > gpurun_out/r4f_bench.jsonl
run() {  # label, bench.py path, VAR=value, bench args...
  local label=$1 bp=$2 ev=$3; shift 3
  env $ev timeout -k 10 200 python $bp "$@" --steps 30 --warmup 10 > gpurun_out/r4f_one.log 2>&1 || { tail -20 gpurun_out/r4f_one.log; return 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/r4f_one.log').read().strip().splitlines()[-1]); print('$label', d['config']['model'], d['ms_per_step'], d['value'])" | tee -a gpurun_out/r4f_bench.jsonl
}
for m in "--model resnet50" "--model resnet50_stage --stage 1 --batch 8" "--model resnet50_stage --stage 2 --batch 8"; do
  run "wpe4-fold" bench.py PDE_BN_FOLD=1 $m || exit 1
  run "wpe4-nofold" bench.py PDE_BN_FOLD=0 $m || exit 1
  run "wpe2-fold" variants/wpe2/bench.py PDE_BN_FOLD=1 $m || exit 1
  run "wpe2-nofold" variants/wpe2/bench.py PDE_BN_FOLD=0 $m || exit 1
done
run "wpe4" bench.py PDE_BN_FOLD=1 --model mlp || exit 1
run "wpe2" variants/wpe2/bench.py PDE_BN_FOLD=1 --model mlp || exit 1
