#!/bin/bash
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/b54
export TMPDIR=/tmp
L="python -u scripts/layer_prof.py --C 100 --N 64 --dtype fp32 --steps 2"
bash scripts/gpu_steps.sh \
 "FEDML_AMD_C1F_WGS64=400 timeout -k 10 300 $L > gpurun_out/b54/w400.txt 2>&1" \
 "FEDML_AMD_C1F_WGS64=800 timeout -k 10 300 $L > gpurun_out/b54/w800.txt 2>&1" \
 "FEDML_AMD_C1F_WGS64=100 timeout -k 10 300 $L > gpurun_out/b54/w100.txt 2>&1" \
 "timeout -k 10 300 $L > gpurun_out/b54/w200.txt 2>&1" \
 "FEDML_AMD_C1F_WGS64=400 timeout -k 10 200 python -u scripts/layer_prof.py --C 13 --N 64 --dtype fp32 --steps 3 > gpurun_out/b54/c13_w400.txt 2>&1" \
 "timeout -k 10 200 python -u scripts/layer_prof.py --C 13 --N 64 --dtype fp32 --steps 3 > gpurun_out/b54/c13_w200.txt 2>&1"
