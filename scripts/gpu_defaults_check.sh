#!/bin/bash
# native tests + the three bench lines after a default change
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
echo "== native tests"; timeout -k 10 600 python -u -m pytest tests/test_native_resnet_fp32_gpu.py tests/test_native_resnet_gpu.py tests/test_native_resnet18_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_def.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_def.log; [ $rc -eq 0 ] || exit $rc
for a in "--steps 8 --warmup 2" "--dtype bf16 --steps 8 --warmup 2" "--preset resnet18_cifar10_10 --dtype bf16 --steps 2 --warmup 1" "--preset resnet18_cifar10_10 --steps 2 --warmup 1"; do
  echo "== bench $a"; timeout -k 10 300 python bench.py $a > gpurun_out/def.log 2>&1 || { tail -3 gpurun_out/def.log; exit 1; }
  tail -1 gpurun_out/def.log >> gpurun_out/def_lines.jsonl; tail -1 gpurun_out/def.log | cut -c1-140
done
