#!/bin/bash
# Round 3, batch n: fp32 3x3 unit-size sweep per channel count (scripts/c3_time.py), then headline A/B of the best.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
out=gpurun_out/c3_px_sweep.txt; : > $out
run() { echo "== $*" >> $out; env "$@" timeout -k 10 120 python scripts/c3_time.py --shapes $SH >> $out 2>&1 || { echo FAIL >> $out; exit 1; }; }
SH=16x32x1 run X=1; SH=16x32x1 run FEDML_AMD_C3_PX16=128; SH=16x32x1 run FEDML_AMD_C3_PX16=512
SH=32x16x1 run X=1; SH=32x16x1 run FEDML_AMD_C3_PX32=128; SH=32x16x1 run FEDML_AMD_C3_PX32=64
SH=64x8x1 run X=1; SH=64x8x1 run FEDML_AMD_C3_PX64=64; SH=64x8x1 run FEDML_AMD_C3_PX64=256
grep -v amdgpu.ids $out
for v in base px base px; do
  if [ $v = px ]; then E="FEDML_AMD_C3_PX32=${PX32:-128}"; else E=X=1; fi
  env $E timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > gpurun_out/b_n_$v.log 2>&1; rc=$?
  echo "$v: $(grep '^{' gpurun_out/b_n_$v.log | cut -c60-140)"; [ $rc -eq 0 ] || exit $rc
done
