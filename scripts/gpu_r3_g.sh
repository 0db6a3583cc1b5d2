#!/bin/bash
# Round 3, batch g: fp32 ResNet-18 preset (bench + rocprofv3 kernel stats), then BASELINE config 5.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --preset resnet18_cifar10_10 --steps 2 --warmup 1 > gpurun_out/b_r18.log 2>&1; rc=$?
grep '^{' gpurun_out/b_r18.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_prof_preset.sh resnet18_cifar10_10 || exit 1
head -25 gpurun_out/prof_resnet18_cifar10_10_summary.txt
bash scripts/gpu_r3_e.sh
