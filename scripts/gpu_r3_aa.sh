#!/bin/bash
# Round 3, batch aa: final PMC table of the fp32 headline and the C=13 / C=100 fp32 layer rooflines.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/layer_prof.py --model resnet56 --C 13 --N 64 --dtype fp32 --steps 3 > gpurun_out/layers_c13.txt 2>&1 || exit 1
timeout -k 10 300 python -u scripts/layer_prof.py --model resnet56 --C 100 --N 64 --dtype fp32 --steps 2 > gpurun_out/layers_c100.txt 2>&1 || exit 1
head -3 gpurun_out/layers_c13.txt; tail -2 gpurun_out/layers_c13.txt | cut -c1-200
PMC_OUT=gpurun_out/pmc_table_final.txt bash scripts/gpu_pmc_r3.sh || exit 1
