#!/bin/bash
# small-grid tile choice of the K-streamed conv kernel: ResNet-18 bf16 A/B
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
export TMPDIR=/tmp
L="python -u scripts/layer_prof.py --C 10 --N 64 --model resnet18 --dtype bf16 --steps 2"
bash scripts/gpu_steps.sh \
 "timeout -k 10 200 $L > gpurun_out/r4_r18_small_0.txt 2>&1" \
 "FEDML_AMD_CONVK_SMALL=512 timeout -k 10 200 $L > gpurun_out/r4_r18_small_512_t2.txt 2>&1" \
 "FEDML_AMD_CONVK_SMALL=512 FEDML_AMD_CONVK_SMALL_TILE=3 timeout -k 10 200 $L > gpurun_out/r4_r18_small_512_t3.txt 2>&1" \
 "FEDML_AMD_CONVK_SMALL=1024 timeout -k 10 200 $L > gpurun_out/r4_r18_small_1024_t2.txt 2>&1" \
 "FEDML_AMD_CONVK_SMALL=1024 FEDML_AMD_CONVK_SMALL_TILE=3 timeout -k 10 200 $L > gpurun_out/r4_r18_small_1024_t3.txt 2>&1"
