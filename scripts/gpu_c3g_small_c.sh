#!/bin/bash
# fp32 3x3 forward / backward-data workgroup target (FEDML_AMD_C3G_WGS) vs clients per GPU
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() {  # wgs C
  FEDML_AMD_C3G_WGS=$1 timeout -k 10 200 python -u scripts/layer_prof.py --dtype fp32 --C $2 > gpurun_out/g$1_c$2.txt 2>&1 || exit 1
  echo "wgs=$1 C=$2 $(grep 'step time' gpurun_out/g$1_c$2.txt | cut -c1-24) fwd $(grep -o 'conv3x3_fwd [0-9.]* ms' gpurun_out/g$1_c$2.txt) bwd $(grep -o 'conv3x3_bwd_data [0-9.]* ms' gpurun_out/g$1_c$2.txt)"
}
run 512 13
run 1024 13
run 2048 13
run 4096 13
run 1024 100
run 4096 100
