#!/bin/bash
# Round-2 first GPU pass: new comm tests first (xGMI one-shot rehearsal, hvd abort), then the whole GPU
# suite, smoke, the default bench and a 2-rank-on-one-GPU rehearsal of the resnet50_pp bench.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() {  # step <name> <timeout> <cmd...>: stop the script on a hard failure (timeout/abort/fault)
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -${TAILN:-15} "gpurun_out/$name.log"
  if [ $rc -gt 1 ]; then exit $rc; fi
  return 0
}
step new_tests 400 python -u -m pytest tests/test_xgmi_gpu.py tests/test_comm_gpu.py tests/test_models_gpu.py -x -v --timeout 150 --timeout-method thread
TAILN=40 step gpu_suite 1000 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread
step smoke 150 python -c "import __graft_entry__ as g; g.smoke()"
step bench_cnn 200 python bench.py --steps 30 --warmup 10
PDE_BACKEND=gloo step bench_pp_rehearsal 400 python bench.py --gpus 2 --model resnet50_pp --steps 3 --warmup 1
step app_ddp_cnn_fused 300 python pytorch_elastic/mnist_ddp_elastic.py 2 5 --model cnn --fused --batch_size 1024 --snapshot_path /tmp/pde_snap.pt
