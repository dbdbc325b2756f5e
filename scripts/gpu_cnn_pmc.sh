#!/bin/bash
# Fused-CNN measurement: tests, phase stamps, bench, then two SQ counter passes over the eager step.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=$(pwd)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -${TAILN:-14} "gpurun_out/$name.log"
  if [ $rc -gt 1 ]; then exit $rc; fi
  return 0
}
step cnn_tests 300 python -u -m pytest tests/test_models_gpu.py -k "cnn" -x -q --timeout 120 --timeout-method thread
step stamps 120 python scripts/cnn_phase_stamps.py
step bench_cnn 200 python bench.py --steps 50 --warmup 10
pass=0
for ctrs in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS" \
            "SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_UNALIGNED_STALL SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES"; do
  pass=$((pass + 1))
  cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $ctrs -d "$R/gpurun_out/pmc_cnn$pass" -o cnn --output-format csv \
    -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-graph > "$R/gpurun_out/pmc_cnn$pass.log" 2>&1
  rc=$?; cd "$R"
  if [ $rc -ne 0 ]; then echo "pmc pass $pass rc=$rc"; tail -5 gpurun_out/pmc_cnn$pass.log; exit $rc; fi
  f=$(find gpurun_out/pmc_cnn$pass -name "*counter_collection.csv" | head -1)
  python3 scripts/pmc_summary.py "$f" 4 | tee gpurun_out/pmc_cnn$pass.txt
done
