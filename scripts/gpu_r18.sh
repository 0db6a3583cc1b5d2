#!/bin/bash
# ResNet-18 wide-channel native path: kernel/step GPU tests, then the config-2 preset at fp32 and bf16
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
echo "== r18 tests"; [ -n "$SKIP18" ] || timeout -k 10 600 python -u -m pytest tests/test_native_resnet18_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r18.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_r18.log; [ $rc -eq 0 ] || exit $rc
echo "== r56 native tests"; timeout -k 10 600 python -u -m pytest tests/test_native_resnet_fp32_gpu.py tests/test_native_resnet_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_q.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_q.log; [ $rc -eq 0 ] || exit $rc
echo "== r18 bf16"; timeout -k 10 400 python bench.py --preset resnet18_cifar10_10 --dtype bf16 --steps 3 --warmup 1 > gpurun_out/bench_r18_bf16.log 2>&1; rc=$?; tail -1 gpurun_out/bench_r18_bf16.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
echo "== r18 fp32"; timeout -k 10 400 python bench.py --preset resnet18_cifar10_10 --steps 2 --warmup 1 > gpurun_out/bench_r18_fp32.log 2>&1; rc=$?; tail -1 gpurun_out/bench_r18_fp32.log | cut -c1-400; exit $rc
