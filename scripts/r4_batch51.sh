#!/bin/bash
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/b51
export TMPDIR=/tmp
bash scripts/gpu_steps.sh \
 "timeout -k 10 300 python -u scripts/layer_prof.py --C 10 --N 64 --model resnet18 --dtype bf16 --steps 2 > gpurun_out/b51/r18b.txt 2>&1" \
 "timeout -k 10 300 python -u scripts/layer_prof.py --C 100 --N 64 --dtype fp32 --steps 2 > gpurun_out/b51/c100.txt 2>&1"
