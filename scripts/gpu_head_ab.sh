#!/bin/bash
# A/B env settings on the fp32 headline (and a numerics check of the last setting)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for e in "$@"; do
  echo "== $e"; env $e timeout -k 10 300 python bench.py --steps 5 --warmup 1 ${BENCH_ARGS} > gpurun_out/ab.log 2>&1 || { tail -3 gpurun_out/ab.log; exit 1; }
  tail -1 gpurun_out/ab.log | cut -c1-150
done
if [ -n "$CHECK_ENV" ]; then
  echo "== fp32 native tests with $CHECK_ENV"; env $CHECK_ENV timeout -k 10 400 python -u -m pytest tests/test_native_resnet_fp32_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_ab.log; exit $rc
fi
