#!/bin/bash
# Round 3, batch p: final PMC table of the fp32 headline + secondary bench lines (13-client share, ResNet-18 fp32/bf16,
# transformer presets fp32).
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
PMC_OUT=gpurun_out/pmc_table_final.txt bash scripts/gpu_pmc_r3.sh || exit 1
b() {  # name args...
  local n=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > gpurun_out/b_p_$n.log 2>&1; local rc=$?
  grep '^{' gpurun_out/b_p_$n.log | cut -c1-160; [ $rc -eq 0 ] || { tail -20 gpurun_out/b_p_$n.log; exit $rc; }
}
b c13 --clients 13 --steps 20 --warmup 3
b r18_fp32 --preset resnet18_cifar10_10 --steps 2 --warmup 1
b r18_bf16 --preset resnet18_cifar10_10 --dtype bf16 --steps 3 --warmup 1
b distil_fp32 --preset distilbert_fedopt_32 --dtype fp32 --steps 3 --warmup 1
b vit_fp32 --preset vit_b16_32 --dtype fp32 --steps 3 --warmup 1

for t in 2 3; do export FEDML_AMD_CONVK_TILE=$t; b r18_bf16_tile$t --preset resnet18_cifar10_10 --dtype bf16 --steps 3 --warmup 1; done; unset FEDML_AMD_CONVK_TILE
for t in 2 3; do export FEDML_AMD_CONVK_TILE=$t; b r18_fp32_tile$t --preset resnet18_cifar10_10 --steps 2 --warmup 1; done; unset FEDML_AMD_CONVK_TILE
timeout -k 10 300 python -u scripts/layer_prof.py --model resnet18 --C 10 --N 64 --dtype bf16 --steps 2 > gpurun_out/r18_bf16_layers.txt 2>&1 || exit 1
head -40 gpurun_out/r18_bf16_layers.txt | cut -c1-130
