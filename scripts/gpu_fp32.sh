#!/bin/bash
# fp32 native path: kernel/step/convergence GPU tests, the bf16 native tests (regression), fp32 + bf16
# headline bench lines, and a rocprofv3 kernel-stats pass of the fp32 headline.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
echo "== fp32 tests"; timeout -k 10 600 python -u -m pytest tests/test_native_resnet_fp32_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_fp32.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_fp32.log; [ $rc -eq 0 ] || exit $rc
echo "== bf16 native tests"; timeout -k 10 600 python -u -m pytest tests/test_native_resnet_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_native.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_native.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
echo "== bench fp32"; timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_fp32.log 2>&1; rc=$?; tail -1 gpurun_out/bench_fp32.log; [ $rc -eq 0 ] || exit $rc
echo "== bench bf16"; timeout -k 10 300 python bench.py --dtype bf16 --steps 10 --warmup 3 > gpurun_out/bench_bf16.log 2>&1; rc=$?; tail -1 gpurun_out/bench_bf16.log; [ $rc -eq 0 ] || exit $rc
if [ "${PROFILE:-1}" = "1" ]; then
  echo "== rocprofv3 fp32"
  R=$GRAFT_REPO_ROOT
  cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_fp32 -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 > $R/gpurun_out/prof_fp32.log 2>&1; rc=$?; tail -2 $R/gpurun_out/prof_fp32.log; exit $rc
fi
