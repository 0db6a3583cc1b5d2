#!/bin/bash
# round 5, call Z16: per-op layer rooflines of ResNet-18 with the weight gradients on the main stream (clean per-op times)
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5z16
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$PWD FEDML_AMD_SIDE_WGRAD=0
timeout -k 10 300 python -u scripts/layer_prof.py --model resnet18 --C 10 --N 64 --dtype fp32 > gpurun_out/r5z16/r18_fp32.txt 2>&1 && \
timeout -k 10 300 python -u scripts/layer_prof.py --model resnet18 --C 10 --N 64 --dtype bf16 > gpurun_out/r5z16/r18_bf16.txt 2>&1
