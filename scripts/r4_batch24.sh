#!/bin/bash
# two-stage LDS pipeline of the K-streamed conv kernel: tests + A/B benches
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_steps.sh \
 "timeout -k 10 600 python -u -m pytest tests/test_native_resnet_gpu.py tests/test_native_resnet18_gpu.py tests/test_native_resnet_fp32_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/r4_t24.log 2>&1" \
 "timeout -k 10 200 python -u bench.py --preset resnet18_cifar10_10 --dtype bf16 --steps 3 --warmup 1 > gpurun_out/r4_r18_bf16_db1.json 2>&1" \
 "FEDML_AMD_CONVK_DB=0 timeout -k 10 200 python -u bench.py --preset resnet18_cifar10_10 --dtype bf16 --steps 3 --warmup 1 > gpurun_out/r4_r18_bf16_db0.json 2>&1" \
 "timeout -k 10 300 python -u bench.py --preset resnet18_cifar10_10 --steps 2 --warmup 1 > gpurun_out/r4_r18_fp32_db1.json 2>&1" \
 "FEDML_AMD_CONVK_DB=0 timeout -k 10 300 python -u bench.py --preset resnet18_cifar10_10 --steps 2 --warmup 1 > gpurun_out/r4_r18_fp32_db0.json 2>&1" \
 "timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r4_head_db1.json 2>&1" \
 "FEDML_AMD_CONVK_DB=0 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r4_head_db0.json 2>&1" \
 "timeout -k 10 300 python -u scripts/layer_prof.py --C 10 --N 64 --model resnet18 --dtype bf16 --steps 2 > gpurun_out/r4_r18_bf16_layers_b24.txt 2>&1"
