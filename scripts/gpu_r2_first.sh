#!/bin/bash
# Round-2 first GPU pass: GPU tests, headline bench (bf16 native), and the torch fp32 batched path for reference.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
echo "== pytest gpu"; timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== bench bf16"; timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_bf16.log 2>&1; rc=$?; tail -1 gpurun_out/bench_bf16.log; [ $rc -eq 0 ] || exit $rc
echo "== bench torch fp32"; FEDML_AMD_NATIVE_CONV=0 timeout -k 10 400 python bench.py --dtype fp32 --steps 2 --warmup 1 > gpurun_out/bench_torch_fp32.log 2>&1; rc=$?; tail -1 gpurun_out/bench_torch_fp32.log; exit $rc
