#!/bin/bash
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/b56
export TMPDIR=/tmp
L="python -u scripts/layer_prof.py --C 100 --N 64 --dtype fp32 --steps 2"
bash scripts/gpu_steps.sh \
 "FEDML_AMD_C3_PX16=128 timeout -k 10 300 $L > gpurun_out/b56/p128.txt 2>&1" \
 "FEDML_AMD_C3_PX16=512 timeout -k 10 300 $L > gpurun_out/b56/p512.txt 2>&1" \
 "FEDML_AMD_C3_PX32=128 timeout -k 10 300 $L > gpurun_out/b56/q128.txt 2>&1" \
 "timeout -k 10 300 $L > gpurun_out/b56/base.txt 2>&1"
