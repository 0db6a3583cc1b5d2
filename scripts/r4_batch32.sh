#!/bin/bash
# pixel-scaled fp32 3x3 workgroup targets: benches (R18 fp32, headline, C13) + bf16 knob sweep on ResNet-18
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/sw32
export TMPDIR=/tmp
L="python -u scripts/layer_prof.py --C 10 --N 64 --model resnet18 --dtype bf16 --steps 2"
bash scripts/gpu_steps.sh \
 "timeout -k 10 300 python -u bench.py --preset resnet18_cifar10_10 --steps 2 --warmup 1 > gpurun_out/sw32/r18_fp32.json 2>&1" \
 "timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > gpurun_out/sw32/c100.json 2>&1" \
 "timeout -k 10 150 python -u bench.py --clients 13 --steps 20 --warmup 3 > gpurun_out/sw32/c13.json 2>&1" \
 "timeout -k 10 200 $L > gpurun_out/sw32/bf_base.txt 2>&1" \
 "FEDML_AMD_C3W_WGS=512 timeout -k 10 200 $L > gpurun_out/sw32/bf_w512.txt 2>&1" \
 "FEDML_AMD_C3W_WGS=1024 timeout -k 10 200 $L > gpurun_out/sw32/bf_w1024.txt 2>&1" \
 "FEDML_AMD_C3G_WGS=1024 timeout -k 10 200 $L > gpurun_out/sw32/bf_g1024.txt 2>&1" \
 "FEDML_AMD_C3G_WGS=4096 timeout -k 10 200 $L > gpurun_out/sw32/bf_g4096.txt 2>&1" \
 "FEDML_AMD_C3_PX64=256 timeout -k 10 200 $L > gpurun_out/sw32/bf_px256.txt 2>&1"
