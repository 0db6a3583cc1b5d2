#!/bin/bash
# ResNet-18 fp32: K-streamed conv tile and wide weight-gradient targets
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/sw38
export TMPDIR=/tmp
L="python -u scripts/layer_prof.py --C 10 --N 64 --model resnet18 --dtype fp32 --steps 2"
bash scripts/gpu_steps.sh \
 "timeout -k 10 200 $L > gpurun_out/sw38/base.txt 2>&1" \
 "FEDML_AMD_CONVK_TILE=2 timeout -k 10 200 $L > gpurun_out/sw38/t2.txt 2>&1" \
 "FEDML_AMD_CONVK_TILE=0 timeout -k 10 200 $L > gpurun_out/sw38/t0.txt 2>&1" \
 "FEDML_AMD_WGW_WGS=1024 timeout -k 10 200 $L > gpurun_out/sw38/wgw1024.txt 2>&1" \
 "FEDML_AMD_WGW_WGS=4096 timeout -k 10 200 $L > gpurun_out/sw38/wgw4096.txt 2>&1" \
 "FEDML_AMD_CONVK_MIN_K=128 timeout -k 10 200 $L > gpurun_out/sw38/mk128.txt 2>&1"
