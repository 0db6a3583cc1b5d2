#!/bin/bash
# ResNet-18 x10: MIOpen batch norm vs ATen native batch norm on the per-client path.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for bn in miopen native miopen native; do
  FEDML_AMD_SEQ_BN=$bn timeout -k 10 600 python -u bench.py --preset resnet18_cifar10_10 --steps 2 --warmup 1 > gpurun_out/bench_r18_$bn.log 2>&1 || { tail -20 gpurun_out/bench_r18_$bn.log; exit 1; }
  echo "bn=$bn $(grep -o '"value": [0-9.]*' gpurun_out/bench_r18_$bn.log) $(grep -o '"final_train_loss": [0-9.]*' gpurun_out/bench_r18_$bn.log)"
done
