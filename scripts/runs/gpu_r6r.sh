#!/bin/bash
# Round-6 R: low-K GEMM (B strip via LDS, grid cap 256): numerics, microbench + write-bandwidth reference,
# ResNet-50 / stage A/B, shape table.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6r_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r6r_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/gemm_lowk_bench.py > gpurun_out/r6r_lowk.jsonl 2>gpurun_out/r6r_err.log || { tail -5 gpurun_out/r6r_err.log; exit 1; }
PDE_GEMM_LOWK=0 timeout -k 10 120 python scripts/gemm_lowk_bench.py >> gpurun_out/r6r_lowk.jsonl 2>>gpurun_out/r6r_err.log || exit 1
cat gpurun_out/r6r_lowk.jsonl
bench() {  # label, args...
  local label=$1; shift
  timeout -k 10 200 python bench.py "$@" > gpurun_out/r6r_$label.log 2>&1 || { tail -5 gpurun_out/r6r_$label.log; return 1; }
  echo "$label $(grep '^{' gpurun_out/r6r_$label.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
}
bench resnet50 --model resnet50 --steps 30 --warmup 10 || exit 1
PDE_GEMM_LOWK=0 bench resnet50_off --model resnet50 --steps 30 --warmup 10 || exit 1
bench resnet50_b --model resnet50 --steps 30 --warmup 10 || exit 1
bench stage1 --model resnet50_stage --stage 1 --batch 8 --steps 40 --warmup 5 || exit 1
PDE_GEMM_LOWK=0 bench stage1_off --model resnet50_stage --stage 1 --batch 8 --steps 40 --warmup 5 || exit 1
bench stage2 --model resnet50_stage --stage 2 --batch 8 --steps 40 --warmup 5 || exit 1
export TMPDIR=/tmp PDE_GEMM_LOG=1 PDE_BENCH_PHASES=0 PDE_BENCH_OVERHEADS=0
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r6r_gs" -o "r" --output-format csv \
  -- python3 "$R/bench.py" --no-graph --steps 3 --warmup 1 --model resnet50 > "$R/gpurun_out/r6r_gs.log" 2>&1 || { echo "trace failed"; exit 1; }
cd "$R"
f=$(find gpurun_out/r6r_gs -name '*kernel_trace.csv' | head -1)
python3 scripts/gemm_shape_table.py gpurun_out/r6r_gs.log "$f" --steps 4 --title "resnet50 b32: GEMM launches of one eager step (low-K path, B strip via LDS)" > gpurun_out/r6r_gemm_shapes.md
sed -n 3p gpurun_out/r6r_gemm_shapes.md; grep lowk gpurun_out/r6r_gemm_shapes.md
