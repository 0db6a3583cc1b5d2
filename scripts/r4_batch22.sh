#!/bin/bash
# C13 share: kernel stats + layer roofline; ResNet-18 layer rooflines (fp32, bf16); transformer glue call sites
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_steps.sh \
 "timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c13 -o c13 -- python3 bench.py --clients 13 --steps 3 --warmup 1 > gpurun_out/r4_c13_prof.log 2>&1" \
 "timeout -k 10 200 python -u scripts/layer_prof.py --C 13 --N 64 --dtype fp32 > gpurun_out/r4_c13_layers.txt 2>&1" \
 "timeout -k 10 300 python -u scripts/layer_prof.py --C 10 --N 64 --model resnet18 --dtype fp32 --steps 2 > gpurun_out/r4_r18_fp32_layers.txt 2>&1" \
 "timeout -k 10 300 python -u scripts/layer_prof.py --C 10 --N 64 --model resnet18 --dtype bf16 --steps 2 > gpurun_out/r4_r18_bf16_layers.txt 2>&1" \
 "timeout -k 10 300 python -u scripts/torch_op_prof.py --preset distilbert_fedopt_32 --stacks aten::fill_,aten::copy_,aten::add_,aten::mul > gpurun_out/r4_distil_ops3.txt 2>&1"
