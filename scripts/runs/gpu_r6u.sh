#!/bin/bash
# Round-6 U: BatchNorm forward: pivot + first-row slab loads batched together.  Numerics (incl. deferred-slab
# bitwise test), stage benches, stage-2 BN grid table.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_bn_sidestream_gpu.py tests/test_bnfold_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r6u_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|Error|passed|failed" gpurun_out/r6u_pytest.log | tail -5
[ $rc -eq 0 ] || exit $rc
bench() {  # label, args...
  local label=$1; shift
  timeout -k 10 200 python bench.py "$@" > gpurun_out/r6u_$label.log 2>&1 || { tail -5 gpurun_out/r6u_$label.log; return 1; }
  echo "$label $(grep '^{' gpurun_out/r6u_$label.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
}
bench stage2 --model resnet50_stage --stage 2 --batch 8 --steps 40 --warmup 5 || exit 1
bench stage1 --model resnet50_stage --stage 1 --batch 8 --steps 40 --warmup 5 || exit 1
bench resnet50 --model resnet50 --steps 30 --warmup 10 || exit 1
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r6u_prof_s2" -o s2 --output-format csv -- python3 "$R/bench.py" \
    --model resnet50_stage --stage 2 --batch 8 --steps 40 --warmup 5 > "$R/gpurun_out/r6u_prof_s2.log" 2>&1 || { echo "profile failed"; exit 1; }
cd "$R"
python3 scripts/bn_grid_table.py gpurun_out/r6u_prof_s2/s2_kernel_trace.csv | tee gpurun_out/r6u_bn_grid_s2.md
python3 scripts/graph_kernel_table.py gpurun_out/r6u_prof_s2/s2_kernel_trace.csv --title "resnet50 stage 2 m8 r6u" --step-kernel k_optim > gpurun_out/r6u_stage2_m8_graph_kernels.md && sed -n 3p gpurun_out/r6u_stage2_m8_graph_kernels.md
