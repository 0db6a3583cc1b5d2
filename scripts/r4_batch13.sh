#!/bin/bash
# BASELINE presets (ResNet-18 fp32/bf16, DistilBERT, ViT), fp32 transformer GEMM micro, torch-op glue attribution
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_steps.sh \
 "timeout -k 10 500 python -u -m pytest tests/test_transformer_f32_gpu.py tests/test_transformer_kernels_gpu.py tests/test_plane_ops_gpu.py tests/test_determinism.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/r4_t13.log 2>&1" \
 "timeout -k 10 300 python -u bench.py --preset mobilenet_cifar10_10 --steps 2 --warmup 1 > gpurun_out/r4_mnet_b13.json 2>&1" \
 "timeout -k 10 120 python -u scripts/tf_gemm_micro.py --check > gpurun_out/r4_tfg1_micro.jsonl 2>&1" \
 "timeout -k 10 300 python -u bench.py --preset distilbert_fedopt_32 --steps 5 --warmup 2 > gpurun_out/r4_distil_b13.json 2>&1" \
 "timeout -k 10 300 python -u bench.py --preset vit_b16_32 --steps 4 --warmup 2 > gpurun_out/r4_vit_b13.json 2>&1" \
 "timeout -k 10 300 python -u bench.py --preset resnet18_cifar10_10 --steps 2 --warmup 1 > gpurun_out/r4_r18_fp32.json 2>&1" \
 "timeout -k 10 300 python -u bench.py --preset resnet18_cifar10_10 --dtype bf16 --steps 3 --warmup 1 > gpurun_out/r4_r18_bf16.json 2>&1" \
 "FEDML_AMD_HIP_GRAPHS=0 timeout -k 10 300 python -u scripts/torch_op_prof.py --preset distilbert_fedopt_32 > gpurun_out/r4_distil_ops.txt 2>&1" \
 "FEDML_AMD_HIP_GRAPHS=0 timeout -k 10 300 python -u scripts/torch_op_prof.py --preset vit_b16_32 > gpurun_out/r4_vit_ops.txt 2>&1"
