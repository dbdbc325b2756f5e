#!/bin/bash
# Round-6 E: stage kernel tables at the reference micro-batch (m = 8, graph mode) + SQ counters of the ResNet-50
# GEMM problems (two counter passes of the same eager command, joined with the GEMM shape log).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p "$R/gpurun_out"
timeout -s KILL 60 rocprofv3 -L > "$R/gpurun_out/r6e_counters_avail.txt" 2>&1 || true
for s in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r6e_prof_s$s" -o s$s --output-format csv -- python3 "$R/bench.py" \
    --model resnet50_stage --stage $s --batch 8 --steps 40 --warmup 5 > "$R/gpurun_out/r6e_prof_s$s.log" 2>&1 || { echo "profile failed"; tail -5 "$R/gpurun_out/r6e_prof_s$s.log"; exit 1; }
  python3 "$R/scripts/graph_kernel_table.py" "$R/gpurun_out/r6e_prof_s$s/s${s}_kernel_trace.csv" --title "resnet50 stage $s m8 r6e" --step-kernel k_optim \
    > "$R/gpurun_out/r6e_stage${s}_m8_graph_kernels.md" && head -30 "$R/gpurun_out/r6e_stage${s}_m8_graph_kernels.md"
done
export PDE_GEMM_LOG=1 PDE_BENCH_PHASES=0 PDE_BENCH_OVERHEADS=0
pass=0
# (the two counter sets of the round-4 CNN passes, proven on this pool: 8 SQ counters each)
for ctrs in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS" \
            "SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_UNALIGNED_STALL SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  pass=$((pass + 1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs -d "$R/gpurun_out/r6e_pmc$pass" -o p --output-format csv \
    -- python3 "$R/bench.py" --no-graph --model resnet50 --steps 2 --warmup 1 > "$R/gpurun_out/r6e_pmc$pass.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pmc pass $pass rc=$rc"; tail -8 "$R/gpurun_out/r6e_pmc$pass.log"; exit 1; fi
done
f1=$(find "$R/gpurun_out/r6e_pmc1" -name "*counter_collection.csv" | head -1)
f2=$(find "$R/gpurun_out/r6e_pmc2" -name "*counter_collection.csv" | head -1)
python3 "$R/scripts/gemm_pmc_table.py" "$R/gpurun_out/r6e_pmc1.log" "$f1" "$f2" --steps 3 --top 8 --title "resnet50 b32 GEMM SQ counters r6e" > "$R/gpurun_out/r6_gemm_sq_counters.md"
head -20 "$R/gpurun_out/r6_gemm_sq_counters.md" | cut -c1-400
# the Horovod-elastic step (AdamW, batch 128): where its 0.05 ms go
unset PDE_GEMM_LOG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r6e_prof_hvde" -o h --output-format csv -- python3 "$R/bench.py" \
  --model hvd_cnn_elastic --steps 200 --warmup 20 > "$R/gpurun_out/r6e_prof_hvde.log" 2>&1 || { echo "hvde profile failed"; tail -5 "$R/gpurun_out/r6e_prof_hvde.log"; exit 1; }
python3 "$R/scripts/graph_kernel_table.py" "$R/gpurun_out/r6e_prof_hvde/h_kernel_trace.csv" --title "hvd_cnn_elastic b128 r6e" --step-kernel k_optim \
  > "$R/gpurun_out/r6e_hvd_cnn_elastic_kernels.md" && head -16 "$R/gpurun_out/r6e_hvd_cnn_elastic_kernels.md"
