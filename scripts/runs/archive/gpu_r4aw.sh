#!/bin/bash
# Round-4 full check AW (final state of the session): the whole GPU test suite, smoke(), and the benches of every model (+ stages, elastic
# world-1 round), saved for profiles/.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r4aw_pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r4aw_pytest.log | tail -12
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4aw_smoke.log 2>&1 || { tail -20 gpurun_out/r4aw_smoke.log; exit 1; }
tail -1 gpurun_out/r4aw_smoke.log
: > gpurun_out/r4aw_bench.jsonl
for m in "cnn" "hvd_cnn" "mlp" "resnet50" "resnet50_stage --stage 1 --batch 8" "resnet50_stage --stage 2 --batch 8" \
         "resnet50_stage --stage 1 --batch 32 --mb-group 4" "resnet50_stage --stage 2 --batch 32 --mb-group 4"; do
  timeout -k 10 200 python bench.py --model $m --steps 30 --warmup 10 > gpurun_out/r4aw_one.log 2>&1 || { tail -20 gpurun_out/r4aw_one.log; exit 1; }
  tail -1 gpurun_out/r4aw_one.log >> gpurun_out/r4aw_bench.jsonl
  tail -1 gpurun_out/r4aw_one.log | cut -c1-220
done
timeout -k 10 200 python bench.py > gpurun_out/r4aw_default.log 2>&1 && tail -1 gpurun_out/r4aw_default.log | cut -c1-300

cd /tmp && export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"
for m in cnn resnet50 mlp; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r4aw_prof_$m" -o $m --output-format csv -- python3 "$R/bench.py" --model $m --steps 40 --warmup 5 > "$R/gpurun_out/r4aw_prof_$m.log" 2>&1 || { echo "profile $m failed"; tail -5 "$R/gpurun_out/r4aw_prof_$m.log"; exit 1; }
  step=k_optim; [ $m = cnn ] && step=k_cnn_reduce
  python3 "$R/scripts/graph_kernel_table.py" "$R/gpurun_out/r4aw_prof_$m/${m}_kernel_trace.csv" --title "$m r4aw" --step-kernel $step > "$R/gpurun_out/r4aw_${m}_graph_kernels.md"
  head -12 "$R/gpurun_out/r4aw_${m}_graph_kernels.md"
done
