#!/bin/bash
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for w in 2048 256 128; do
  for c in 50 25 13; do
    FEDML_AMD_C3W_WGS=$w timeout -k 10 300 python -u bench.py --clients $c --steps 3 --warmup 1 > gpurun_out/bench_w$w_c$c.log 2>&1 || { tail -20 gpurun_out/bench_w$w_c$c.log; exit 1; }
    echo "wgs=$w C=$c $(grep -o '"value": [0-9.]*' gpurun_out/bench_w$w_c$c.log)"
  done
done
