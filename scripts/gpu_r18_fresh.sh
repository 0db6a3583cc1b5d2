#!/bin/bash
# ResNet-18 x10 preset on a fresh box (cold MIOpen caches), twice; FIND=0 reproduces heuristic mode.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 600 python -u bench.py --preset resnet18_cifar10_10 --steps 2 --warmup 1 > gpurun_out/bench_r18_run$i.log 2>&1 || { tail -20 gpurun_out/bench_r18_run$i.log; exit 1; }
  echo "run $i $(grep -o '"value": [0-9.]*' gpurun_out/bench_r18_run$i.log)"
done
