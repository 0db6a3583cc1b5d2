#!/bin/bash
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/b47
export TMPDIR=/tmp
bash scripts/gpu_steps.sh \
 "FEDML_AMD_CONVK_MIN_K=128 timeout -k 10 200 python -u bench.py --preset resnet18_cifar10_10 --dtype bf16 --steps 3 --warmup 1 > gpurun_out/b47/rb128.json 2>&1" \
 "timeout -k 10 200 python -u bench.py --preset resnet18_cifar10_10 --dtype bf16 --steps 3 --warmup 1 > gpurun_out/b47/rb256.json 2>&1" \
 "FEDML_AMD_CONVK_MIN_K=128 timeout -k 10 300 python -u bench.py --preset resnet18_cifar10_10 --steps 2 --warmup 1 > gpurun_out/b47/rf128.json 2>&1" \
 "timeout -k 10 300 python -u bench.py --preset resnet18_cifar10_10 --steps 2 --warmup 1 > gpurun_out/b47/rf256.json 2>&1" \
 "FEDML_AMD_CONVK_MIN_K=128 timeout -k 10 200 python -u bench.py --preset mobilenet_cifar10_10 --steps 2 --warmup 1 > gpurun_out/b47/m128.json 2>&1" \
 "timeout -k 10 200 python -u bench.py --preset mobilenet_cifar10_10 --steps 2 --warmup 1 > gpurun_out/b47/m256.json 2>&1" \
 "FEDML_AMD_CONVK_MIN_K=128 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --dtype bf16 > gpurun_out/b47/hb128.json 2>&1" \
 "timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --dtype bf16 > gpurun_out/b47/hb256.json 2>&1"
