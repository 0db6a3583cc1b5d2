#!/bin/bash
# 13-client share: 3x3 workgroup targets
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/sw37
export TMPDIR=/tmp
L="python -u scripts/layer_prof.py --C 13 --N 64 --dtype fp32 --steps 3"
bash scripts/gpu_steps.sh \
 "timeout -k 10 200 $L > gpurun_out/sw37/base.txt 2>&1" \
 "FEDML_AMD_C3W_WGS=512 timeout -k 10 200 $L > gpurun_out/sw37/w512.txt 2>&1" \
 "FEDML_AMD_C3W_WGS=1024 timeout -k 10 200 $L > gpurun_out/sw37/w1024.txt 2>&1" \
 "FEDML_AMD_C3G_WGS=1024 timeout -k 10 200 $L > gpurun_out/sw37/g1024.txt 2>&1" \
 "FEDML_AMD_C3G_WGS=256 timeout -k 10 200 $L > gpurun_out/sw37/g256.txt 2>&1" \
 "FEDML_AMD_WGW_WGS=1024 timeout -k 10 200 $L > gpurun_out/sw37/wgw1024.txt 2>&1"
