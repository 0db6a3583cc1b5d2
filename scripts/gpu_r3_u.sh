#!/bin/bash
# Round 3, batch u: knob sweep at the 13-client share (the per-GPU work of the 8-GPU headline run).
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
out=gpurun_out/knob_sweep_c13.txt; : > $out
for v in X=1 FEDML_AMD_CONV_WGS=256 FEDML_AMD_CONV_WGS=512 FEDML_AMD_CONV_WGS=2048 FEDML_AMD_C1F_PPW=128 \
         FEDML_AMD_C1F_PPW=256 FEDML_AMD_C1_PPW=256 FEDML_AMD_C1_PPW=512 FEDML_AMD_C3G_WGS=256 FEDML_AMD_C3G_WGS=1024 \
         FEDML_AMD_C3W_WGS=128 FEDML_AMD_C3W_WGS=384 FEDML_AMD_C3_PX16=128 FEDML_AMD_C3_PX64=64 X=2; do
  env $v timeout -k 10 200 python -u bench.py --clients 13 --steps 20 --warmup 3 > gpurun_out/b_u.log 2>&1; rc=$?
  echo "$v $(grep '^{' gpurun_out/b_u.log | cut -c60-110)" | tee -a $out; [ $rc -eq 0 ] || exit $rc
done
