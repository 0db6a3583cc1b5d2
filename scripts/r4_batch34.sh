#!/bin/bash
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_steps.sh \
 "timeout -k 10 300 python -u scripts/torch_op_prof.py --preset vit_b16_32 --dtype bf16 --stacks '' --shapes aten::copy_,aten::fill_,aten::add_,aten::mul --rows 30 > gpurun_out/r4_vit_bf16_ops.txt 2>&1" \
 "timeout -k 10 300 python -u scripts/torch_op_prof.py --preset distilbert_fedopt_32 --dtype bf16 --stacks '' --shapes aten::copy_,aten::fill_,aten::add_,aten::mul --rows 30 > gpurun_out/r4_distil_bf16_ops.txt 2>&1"
