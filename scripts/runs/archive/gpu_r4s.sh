#!/bin/bash
# Round-4 check S: per-phase SQ counters of the fused CNN kernel (kernel prefixes, scripts/cnn_phase_pmc.py).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
pass=0
for ctrs in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS" \
            "SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_UNALIGNED_STALL SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  pass=$((pass + 1))
  cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $ctrs -d "$R/gpurun_out/r4s_pmc$pass" -o cnn --output-format csv \
    -- python3 "$R/scripts/cnn_phase_pmc.py" > "$R/gpurun_out/r4s_pmc$pass.log" 2>&1
  rc=$?; cd "$R"
  if [ $rc -ne 0 ]; then echo "pmc pass $pass rc=$rc"; tail -5 gpurun_out/r4s_pmc$pass.log; exit $rc; fi
  f=$(find gpurun_out/r4s_pmc$pass -name "*counter_collection.csv" | head -1)
  python3 scripts/pmc_summary.py "$f" --phases | tee gpurun_out/r4s_pmc$pass.txt
done
