#!/bin/bash
# headline + ResNet-18 bf16 + ViT fp32 kernel statistics (rocprofv3 --stats, csv)
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
cd /tmp
bash $R/scripts/gpu_steps.sh \
 "timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_head4 -o run -- python3 $R/bench.py --steps 2 --warmup 1 > $R/gpurun_out/prof_head4.log 2>&1" \
 "timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r18bf4 -o run -- python3 $R/bench.py --preset resnet18_cifar10_10 --dtype bf16 --steps 1 --warmup 1 > $R/gpurun_out/prof_r18bf4.log 2>&1" \
 "timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_vit4 -o run -- python3 $R/bench.py --preset vit_b16_32 --steps 2 --warmup 1 > $R/gpurun_out/prof_vit4.log 2>&1"
