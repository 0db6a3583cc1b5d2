#!/bin/bash
# full GPU suite (no -x: every failure listed), fp32 transformer GEMM micro, ResNet-18 presets, glue attribution
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_steps.sh \
 "timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/r4_gpu_suite_b15.log 2>&1" \
 "timeout -k 10 120 python -u scripts/tf_gemm_micro.py --check > gpurun_out/r4_tfg1_micro.jsonl 2>&1" \
 "timeout -k 10 200 python -u bench.py --preset resnet18_cifar10_10 --steps 2 --warmup 1 > gpurun_out/r4_r18_fp32.json 2>&1" \
 "timeout -k 10 200 python -u bench.py --preset resnet18_cifar10_10 --dtype bf16 --steps 3 --warmup 1 > gpurun_out/r4_r18_bf16.json 2>&1" \
 "FEDML_AMD_HIP_GRAPHS=0 timeout -k 10 200 python -u scripts/torch_op_prof.py --preset distilbert_fedopt_32 > gpurun_out/r4_distil_ops.txt 2>&1"
