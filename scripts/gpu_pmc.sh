#!/bin/bash
# One rocprofv3 PMC pass (SQ block only, 7 counters) over a short eager bench run.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp PYTHONUNBUFFERED=1
m=${1:-resnet50}
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES -d "$R/gpurun_out/pmc_$m" -o "$m" \
  --output-format csv -- python3 "$R/bench.py" --model "$m" --steps 2 --warmup 1 --no-graph > "$R/gpurun_out/pmc_$m.log" 2>&1
rc=$?; tail -3 "$R/gpurun_out/pmc_$m.log"; exit $rc
