#!/bin/bash
# round 5, call Z1: XCD-aware block order of the wide weight-gradient kernel (A/B: microbench + ResNet-18 preset)
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5z1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
B="python -u bench.py --preset resnet18_cifar10_10 --steps 3 --warmup 1"
bash scripts/gpu_steps.sh \
 "timeout -k 10 200 python -u scripts/mb_convk.py bf16 > gpurun_out/r5z1/mb_xcd1.txt 2>&1" \
 "FEDML_AMD_WGW_XCD=0 timeout -k 10 200 python -u scripts/mb_convk.py bf16 > gpurun_out/r5z1/mb_xcd0.txt 2>&1" \
 "timeout -k 10 300 $B --dtype bf16 > gpurun_out/r5z1/r18_bf16_xcd1.txt 2>&1" \
 "FEDML_AMD_WGW_XCD=0 timeout -k 10 300 $B --dtype bf16 > gpurun_out/r5z1/r18_bf16_xcd0.txt 2>&1" \
 "timeout -k 10 300 $B --dtype fp32 > gpurun_out/r5z1/r18_fp32_xcd1.txt 2>&1" \
 "FEDML_AMD_WGW_XCD=0 timeout -k 10 300 $B --dtype fp32 > gpurun_out/r5z1/r18_fp32_xcd0.txt 2>&1"
