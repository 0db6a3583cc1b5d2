#!/bin/bash
# parameter sweep of the fp32 3x3 kernels (unit size, workgroup targets) with scripts/c3_time.py
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/c3_sweep.txt; : > $out
run() { echo "== $*" >> $out; env "$@" timeout -k 10 120 python scripts/c3_time.py >> $out 2>&1 || { echo FAIL >> $out; }; }
run X=1
for px in 64 128 256 512 1024; do run FEDML_AMD_C3_PX=$px; done
for w in 512 1024 4096 8192; do run FEDML_AMD_C3G_WGS=$w; done
for w in 128 512 1024 2048; do run FEDML_AMD_C3W_WGS=$w; done
tail -3 $out
