#!/bin/bash
# native kernel/step GPU tests + fp32/bf16 headline bench lines
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
echo "== native tests"; timeout -k 10 600 python -u -m pytest tests/test_native_resnet_fp32_gpu.py tests/test_native_resnet_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_q.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_q.log; [ $rc -eq 0 ] || exit $rc
echo "== bench fp32"; timeout -k 10 400 python bench.py --steps 8 --warmup 2 > gpurun_out/bench_q.log 2>&1; rc=$?; tail -1 gpurun_out/bench_q.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
echo "== bench bf16"; timeout -k 10 300 python bench.py --dtype bf16 --steps 8 --warmup 2 > gpurun_out/bench_q2.log 2>&1; rc=$?; tail -1 gpurun_out/bench_q2.log | cut -c1-300; exit $rc
