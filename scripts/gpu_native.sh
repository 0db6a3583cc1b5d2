#!/bin/bash
# native conv path: numerics test, then bench
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
echo "== native tests"; timeout -k 10 600 python -m pytest tests/test_native_resnet_gpu.py -x -q ${PYTEST_ARGS} > gpurun_out/pytest_native.log 2>&1; rc=$?; tail -30 gpurun_out/pytest_native.log; [ $rc -eq 0 ] || exit $rc
echo "== bench"; timeout -k 10 900 python bench.py ${BENCH_ARGS:---steps 2 --warmup 1} > gpurun_out/bench.log 2>&1; rc=$?; tail -3 gpurun_out/bench.log; exit $rc
