#!/bin/bash
# Round-6 D2: gather / elastic tests, entry scripts, elastic fault bench; then the pp2 x dp2 diagnostic (eager,
# per-phase syncs, short waits) that locates the cross-rank wait of the failed rehearsal.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gather_counter_gpu.py tests/test_elastic_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r6d_pytest.log 2>&1 || { tail -40 gpurun_out/r6d_pytest.log; exit 1; }
tail -6 gpurun_out/r6d_pytest.log
timeout -k 10 600 python scripts/entry_scripts_measure.py gpurun_out/r6_entry_scripts.jsonl > gpurun_out/r6d_entry.log 2>&1 || { tail -40 gpurun_out/r6d_entry.log; exit 1; }
cat gpurun_out/r6d_entry.log
timeout -k 10 600 python bench.py --model elastic_cnn --gpus 2 --scale-to 1 --fault-at 300 --steps 100 --warmup 20 > gpurun_out/r6d_elastic_fault.jsonl 2> gpurun_out/r6d_elastic_fault.err || { tail -30 gpurun_out/r6d_elastic_fault.err; exit 1; }
tail -3 gpurun_out/r6d_elastic_fault.jsonl | cut -c1-1800
PDE_BACKEND=gloo PDE_P2P_TIMEOUT_S=15 PDE_XGMI_TIMEOUT_S=15 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 --master-addr 127.0.0.1 --master-port 29611 scripts/diag_pipe_dp.py 1f1b graph > gpurun_out/r6d_diag.log 2>&1
echo "diag rc=$?"
grep "^\[" gpurun_out/r6d_diag.log | head -60
