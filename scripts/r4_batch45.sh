#!/bin/bash
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/b45
export TMPDIR=/tmp
L="python -u scripts/layer_prof.py --C 100 --N 64 --dtype fp32 --steps 2"
bash scripts/gpu_steps.sh \
 "FEDML_AMD_CONVK_MIN_K=64 timeout -k 10 300 $L > gpurun_out/b45/mk64.txt 2>&1" \
 "FEDML_AMD_CONVK_MIN_K=128 timeout -k 10 300 $L > gpurun_out/b45/mk128.txt 2>&1" \
 "timeout -k 10 300 $L > gpurun_out/b45/base.txt 2>&1"
