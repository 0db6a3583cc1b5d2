#!/bin/bash
# GPU session C: per-client path test + ResNet-18 preset bench + kernel profile.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
PYTHONPATH=$PWD timeout -k 10 300 python -u scripts/mb_resnet18_streams.py graph_streams 2>&1 | grep -v amdgpu.ids
timeout -k 10 400 python -u bench.py --preset resnet18_cifar10_10 --steps 2 --warmup 1 > gpurun_out/bench_resnet18_cifar10_10.log 2>&1 || { tail -30 gpurun_out/bench_resnet18_cifar10_10.log; exit 1; }
tail -1 gpurun_out/bench_resnet18_cifar10_10.log
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r18 -o r18 --output-format csv -- python3 bench.py --preset resnet18_cifar10_10 --steps 1 --warmup 1 > gpurun_out/prof_r18.log 2>&1 || { tail -20 gpurun_out/prof_r18.log; exit 1; }
find gpurun_out/prof_r18 -type f ! -name "*stats.csv" -delete; find gpurun_out/prof_r18 -type f
