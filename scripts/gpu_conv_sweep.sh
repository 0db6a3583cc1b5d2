#!/bin/bash
# Sweep the generic conv kernels' workgroup target (tiles per wave) at 100 and 13 clients.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for w in 2048 1024 4096 512; do
  for c in 100 13; do
    FEDML_AMD_CONV_WGS=$w timeout -k 10 300 python -u bench.py --clients $c --steps 3 --warmup 1 > gpurun_out/bench_cw$w_c$c.log 2>&1 || { tail -20 gpurun_out/bench_cw$w_c$c.log; exit 1; }
    echo "convwgs=$w C=$c $(grep -o '"value": [0-9.]*' gpurun_out/bench_cw$w_c$c.log)"
  done
done
