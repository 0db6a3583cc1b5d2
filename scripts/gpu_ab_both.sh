#!/bin/bash
# A/B env settings on the ResNet-18 preset (bf16) and the fp32 headline
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for e in "$@"; do
  echo "== $e"
  env $e timeout -k 10 300 python bench.py --preset resnet18_cifar10_10 --dtype bf16 --steps 2 --warmup 1 > gpurun_out/ab.log 2>&1 || { tail -3 gpurun_out/ab.log; exit 1; }
  tail -1 gpurun_out/ab.log | cut -c1-150
  env $e timeout -k 10 300 python bench.py --steps 4 --warmup 1 > gpurun_out/ab2.log 2>&1 || { tail -3 gpurun_out/ab2.log; exit 1; }
  tail -1 gpurun_out/ab2.log | cut -c1-150
done
