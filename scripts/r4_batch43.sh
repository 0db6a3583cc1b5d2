#!/bin/bash
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/b43
export TMPDIR=/tmp
L="python -u scripts/layer_prof.py --C 100 --N 64 --dtype fp32 --steps 2"
bash scripts/gpu_steps.sh \
 "FEDML_AMD_C3W_WGS=1024 timeout -k 10 300 $L > gpurun_out/b43/w1024.txt 2>&1" \
 "FEDML_AMD_C3W_WGS=4096 timeout -k 10 300 $L > gpurun_out/b43/w4096.txt 2>&1" \
 "FEDML_AMD_C3G_WGS=4096 timeout -k 10 300 $L > gpurun_out/b43/g4096.txt 2>&1"
