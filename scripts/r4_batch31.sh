#!/bin/bash
# ResNet-18 fp32 3x3 tile-kernel knobs (64 channels at 32²): output slice, unit size, workgroup targets
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/sw31
export TMPDIR=/tmp
L="python -u scripts/layer_prof.py --C 10 --N 64 --model resnet18 --dtype fp32 --steps 2"
bash scripts/gpu_steps.sh \
 "timeout -k 10 200 $L > gpurun_out/sw31/base.txt 2>&1" \
 "FEDML_AMD_C3W_WGS=512 timeout -k 10 200 $L > gpurun_out/sw31/w512.txt 2>&1" \
 "FEDML_AMD_C3W_WGS=1024 timeout -k 10 200 $L > gpurun_out/sw31/w1024.txt 2>&1" \
 "FEDML_AMD_C3W_WGS=2048 timeout -k 10 200 $L > gpurun_out/sw31/w2048.txt 2>&1" \
 "FEDML_AMD_C3_N64=32 timeout -k 10 200 $L > gpurun_out/sw31/n32.txt 2>&1" \
 "FEDML_AMD_C3_PX64=64 timeout -k 10 200 $L > gpurun_out/sw31/px64.txt 2>&1" \
 "FEDML_AMD_C3_PX64=256 timeout -k 10 200 $L > gpurun_out/sw31/px256.txt 2>&1" \
 "FEDML_AMD_C3G_WGS=1024 timeout -k 10 200 $L > gpurun_out/sw31/g1024.txt 2>&1" \
 "FEDML_AMD_C3G_WGS=4096 timeout -k 10 200 $L > gpurun_out/sw31/g4096.txt 2>&1"
