#!/bin/bash
# materialised relu(bn(x)) for the wide weight-gradient kernel: tests + ResNet-18 A/B
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/b40
export TMPDIR=/tmp
bash scripts/gpu_steps.sh \
 "timeout -k 10 600 python -u -m pytest tests/test_native_resnet18_gpu.py tests/test_native_resnet_gpu.py tests/test_native_resnet_fp32_gpu.py tests/test_determinism.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/b40/tests.log 2>&1" \
 "timeout -k 10 200 python -u bench.py --preset resnet18_cifar10_10 --dtype bf16 --steps 3 --warmup 1 > gpurun_out/b40/bf_act1.json 2>&1" \
 "FEDML_AMD_WGW_ACT=0 timeout -k 10 200 python -u bench.py --preset resnet18_cifar10_10 --dtype bf16 --steps 3 --warmup 1 > gpurun_out/b40/bf_act0.json 2>&1" \
 "timeout -k 10 300 python -u bench.py --preset resnet18_cifar10_10 --steps 2 --warmup 1 > gpurun_out/b40/f_act1.json 2>&1" \
 "FEDML_AMD_WGW_ACT=0 timeout -k 10 300 python -u bench.py --preset resnet18_cifar10_10 --steps 2 --warmup 1 > gpurun_out/b40/f_act0.json 2>&1"
