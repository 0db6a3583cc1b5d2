#!/bin/bash
# fp32 64-channel 3x3 layers: output channels per workgroup (FEDML_AMD_C3_N64 16 | 32) and unit size
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() {  # name C env...
  n=$1; c=$2; shift 2
  env "$@" timeout -k 10 200 python -u scripts/layer_prof.py --dtype fp32 --C $c > gpurun_out/n_$n.txt 2>&1 || exit 1
  echo "$n $(grep 'step time' gpurun_out/n_$n.txt | cut -c1-24) | $(grep '64->64 s1 @8\|64<-64 s1 @8' gpurun_out/n_$n.txt | awk '{print $1, $(NF-3), $NF}' | tr '\n' ' ')"
}
run base100 100 FEDML_AMD_C3_N64=16
run n32_100 100 FEDML_AMD_C3_N64=32
run n32px64_100 100 FEDML_AMD_C3_N64=32 FEDML_AMD_C3_PX=64
run base13 13 FEDML_AMD_C3_N64=16
run n32_13 13 FEDML_AMD_C3_N64=32
