#!/bin/bash
# Per-client conv path: bf16 channels-last conv-weight shadow vs autocast casts (test + ResNet-18 A/B).
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_native_resnet_gpu.py -k "shadow or multistream" -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_shadow.log 2>&1 || { tail -30 gpurun_out/pt_shadow.log; exit 1; }
tail -1 gpurun_out/pt_shadow.log
for sh in 1 0 1 0; do
  FEDML_AMD_SEQ_CONV_SHADOW=$sh timeout -k 10 600 python -u bench.py --preset resnet18_cifar10_10 --steps 2 --warmup 1 > gpurun_out/bench_r18_sh$sh.log 2>&1 || { tail -20 gpurun_out/bench_r18_sh$sh.log; exit 1; }
  echo "shadow=$sh $(grep -o '"value": [0-9.]*' gpurun_out/bench_r18_sh$sh.log) $(grep -o '"final_train_loss": [0-9.]*' gpurun_out/bench_r18_sh$sh.log)"
done
