#!/bin/bash
# fp32 3x3 weight-gradient workgroup target vs clients per GPU (the 8-GPU share of the headline is 13 clients)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() {  # wgs C
  FEDML_AMD_C3W_WGS=$1 timeout -k 10 200 python -u scripts/layer_prof.py --dtype fp32 --C $2 > gpurun_out/w$1_c$2.txt 2>&1 || exit 1
  echo "wgs=$1 C=$2 $(grep 'step time' gpurun_out/w$1_c$2.txt | cut -c1-24) wgrad $(grep -o 'conv3x3_wgrad [0-9.]* ms' gpurun_out/w$1_c$2.txt)"
}
run 256 13
run 512 13
run 1024 13
run 512 50
run 1024 50
run 2048 50
run 1024 100
