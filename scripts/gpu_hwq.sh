#!/bin/bash
# ResNet-18 x10 preset vs the number of HIP hardware queues (the per-client graph branches run on
# forked streams; HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues).
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 400 python -u bench.py --preset resnet18_cifar10_10 --steps 2 --warmup 1 > gpurun_out/bench_r18_q$q.log 2>&1 || { tail -20 gpurun_out/bench_r18_q$q.log; exit 1; }
  echo "hwq=$q $(grep -o '"value": [0-9.]*' gpurun_out/bench_r18_q$q.log)"
done
