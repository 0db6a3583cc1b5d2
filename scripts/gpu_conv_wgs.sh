#!/bin/bash
# generic conv workgroup-target sweep on the fp32 headline
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/conv_wgs.txt; : > $out
for w in 256 512 1024 2048 4096; do
  echo "== FEDML_AMD_CONV_WGS=$w" >> $out
  FEDML_AMD_CONV_WGS=$w timeout -k 10 300 python bench.py --steps 3 --warmup 1 2>/dev/null | tail -1 | cut -c1-200 >> $out || exit 1
done
cat $out
