#!/bin/bash
# Round-4 check M: write-through BatchNorm outputs (PDE_BN_WT) on top of the write-through GEMM epilogues --
# BN kernel tests, then ResNet-50 / stage benches A/B.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_bnfold_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r4m_pytest.log 2>&1 || { tail -30 gpurun_out/r4m_pytest.log; exit 1; }
tail -1 gpurun_out/r4m_pytest.log
: > gpurun_out/r4m_bench.txt
run() {
  local label=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 200 python bench.py "$@" > gpurun_out/r4m_one.log 2>&1 || { tail -20 gpurun_out/r4m_one.log; return 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4m_one.log').read().strip().splitlines()[-1]); print('$label', d['config']['model'], d['config'].get('stage'), d['ms_per_step'], d['value'])" | tee -a gpurun_out/r4m_bench.txt
}
for rep in 1 2; do
  for cfg in "PDE_BN_WT=0" "PDE_BN_WT=1" "PDE_BN_WT=1 PDE_GEMM_WT=0"; do
    run "$cfg" $cfg -- --model resnet50 --steps 30 --warmup 10 || exit 1
    run "$cfg" $cfg -- --model resnet50_stage --stage 1 --batch 8 --steps 30 --warmup 10 || exit 1
    run "$cfg" $cfg -- --model resnet50_stage --stage 2 --batch 8 --steps 30 --warmup 10 || exit 1
  done
done
# MLP: bytes fetched / written per kernel (two counter passes: FETCH_SIZE and WRITE_SIZE need 3 + 2 TCC counters)
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats -d "$R/gpurun_out/r4m_pmc_fetch" -o mlp --output-format csv -- python3 "$R/bench.py" --model mlp --steps 20 --warmup 5 > "$R/gpurun_out/r4m_pmc_fetch.log" 2>&1 || { tail -5 "$R/gpurun_out/r4m_pmc_fetch.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats -d "$R/gpurun_out/r4m_pmc_write" -o mlp --output-format csv -- python3 "$R/bench.py" --model mlp --steps 20 --warmup 5 > "$R/gpurun_out/r4m_pmc_write.log" 2>&1 || { tail -5 "$R/gpurun_out/r4m_pmc_write.log"; exit 1; }
ls -R "$R/gpurun_out/r4m_pmc_fetch" | head -20
