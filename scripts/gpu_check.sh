#!/bin/bash
# First GPU check: kernel tests, models, smoke, short bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc   # 1 = test failures: still run smoke/bench
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -5 || exit 1
timeout -k 10 200 python bench.py --steps 50 --warmup 10 2>&1 | tail -3 || exit 1
timeout -k 10 200 python bench.py --model mlp --steps 50 --warmup 10 2>&1 | tail -3 || exit 1
timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 3 2>&1 | tail -3 || exit 1
R=$(pwd)
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_cnn -o cnn --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 > $R/gpurun_out/prof_cnn.log 2>&1 || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_resnet -o resnet --output-format csv -- python3 $R/bench.py --model resnet50 --steps 5 --warmup 2 > $R/gpurun_out/prof_resnet.log 2>&1 || exit 1
echo PROFILES_DONE
