#!/bin/bash
# residual / GELU links active on the fp32 engine path + fused bias gradient: tests, presets, glue profile
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_steps.sh \
 "timeout -k 10 400 python -u -m pytest tests/test_transformer_f32_gpu.py tests/test_transformer_kernels_gpu.py tests/test_determinism.py tests/test_apis_gpu.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/r4_t21.log 2>&1" \
 "timeout -k 10 150 python -u bench.py --preset vit_b16_32 --steps 4 --warmup 2 > gpurun_out/r4_vit_b21.json 2>&1" \
 "timeout -k 10 150 python -u bench.py --preset distilbert_fedopt_32 --steps 5 --warmup 2 > gpurun_out/r4_distil_b21.json 2>&1" \
 "timeout -k 10 200 python -u bench.py --preset resnet18_cifar10_10 --dtype bf16 --steps 3 --warmup 1 > gpurun_out/r4_r18_bf16_b21.json 2>&1" \
 "timeout -k 10 300 python -u scripts/torch_op_prof.py --preset vit_b16_32 --stacks '' > gpurun_out/r4_vit_ops3.txt 2>&1"
