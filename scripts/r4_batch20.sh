#!/bin/bash
# wide weight-gradient workgroup target sweep (gx = 1 → direct arena writes, no atomics / scatter) on ResNet-18
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
export TMPDIR=/tmp
steps=()
for t in 2048 1024 512; do
  steps+=("FEDML_AMD_WGW_WGS=$t timeout -k 10 200 python -u bench.py --preset resnet18_cifar10_10 --dtype bf16 --steps 3 --warmup 1 > gpurun_out/r4_r18_bf16_wgw$t.json 2>&1")
done
for t in 2048 512; do
  steps+=("FEDML_AMD_WGW_WGS=$t timeout -k 10 200 python -u bench.py --preset resnet18_cifar10_10 --steps 2 --warmup 1 > gpurun_out/r4_r18_fp32_wgw$t.json 2>&1")
done
steps+=("FEDML_AMD_WGW_WGS=512 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r4_c100_wgw512.json 2>&1")
steps+=("timeout -k 10 300 python -u scripts/torch_op_prof.py --preset vit_b16_32 --trace-dtoh --stacks '' > gpurun_out/r4_vit_dtoh.txt 2>&1")
bash scripts/gpu_steps.sh "${steps[@]}"
