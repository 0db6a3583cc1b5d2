#!/bin/bash
# ResNet-18 preset A/B over env settings (bf16 unless DT set)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
DT=${DT:-bf16}
for e in "$@"; do
  echo "== $e"; env $e timeout -k 10 300 python bench.py --preset resnet18_cifar10_10 --dtype $DT --steps 2 --warmup 1 > gpurun_out/ab.log 2>&1; rc=$?; tail -1 gpurun_out/ab.log | cut -c1-190; [ $rc -eq 0 ] || exit $rc
done
