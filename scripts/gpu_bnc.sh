#!/bin/bash
# Fused channels-last BN(+residual+ReLU) kernels: numerics tests, then ResNet-18 x10 A/B vs MIOpen BN.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_bn_ops_gpu.py tests/test_native_resnet_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/pt_bnc.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/pt_bnc.log | tail -20; }
tail -1 gpurun_out/pt_bnc.log
for bn in 1 0 1 0; do
  FEDML_AMD_BNC=$bn timeout -k 10 600 python -u bench.py --preset resnet18_cifar10_10 --steps 2 --warmup 1 > gpurun_out/bench_r18_bnc$bn.log 2>&1 || { tail -20 gpurun_out/bench_r18_bnc$bn.log; exit 1; }
  echo "bnc=$bn $(grep -o '"value": [0-9.]*' gpurun_out/bench_r18_bnc$bn.log) $(grep -o '"final_train_loss": [0-9.]*' gpurun_out/bench_r18_bnc$bn.log)"
done
