#!/bin/bash
# python-side tile knobs of the native ResNet step at the 13-client share (generic conv WG target, 1x1 fused
# backward pixels per workgroup) — per-step layer profile
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() {  # name env...
  n=$1; shift
  env "$@" timeout -k 10 200 python -u scripts/layer_prof.py --dtype fp32 --C 13 > gpurun_out/k_$n.txt 2>&1 || exit 1
  echo "$n $(grep 'step time' gpurun_out/k_$n.txt | cut -c1-24) $(grep -o -- '-- by op:.*' gpurun_out/k_$n.txt | cut -c1-150)"
}
run base FEDML_AMD_CONV_WGS=1024
run cw512 FEDML_AMD_CONV_WGS=512
run cw2048 FEDML_AMD_CONV_WGS=2048
run cw4096 FEDML_AMD_CONV_WGS=4096
run c1f256 FEDML_AMD_C1F_PPW=256
run c1f1024 FEDML_AMD_C1F_PPW=1024
