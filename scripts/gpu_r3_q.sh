#!/bin/bash
# Round 3, batch q: re-tune the workgroup/unit knobs of the fp32 headline after the kernel changes (bench lines per
# variant, same box).
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
out=gpurun_out/knob_sweep.txt; : > $out
for v in X=1 FEDML_AMD_CONV_WGS=512 FEDML_AMD_CONV_WGS=2048 FEDML_AMD_C1F_PPW=256 FEDML_AMD_C1F_PPW=1024 \
         FEDML_AMD_C1_PPW=1024 FEDML_AMD_C3W_WGS=1024 FEDML_AMD_C3W_WGS=4096 FEDML_AMD_C3G_WGS=1024 \
         FEDML_AMD_C3G_WGS=4096 X=2; do
  env $v timeout -k 10 200 python -u bench.py --steps 6 --warmup 2 > gpurun_out/b_q.log 2>&1; rc=$?
  echo "$v $(grep '^{' gpurun_out/b_q.log | cut -c60-110)" | tee -a $out; [ $rc -eq 0 ] || exit $rc
done
