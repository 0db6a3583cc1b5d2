#!/bin/bash
# Native ResNet path: numerics tests + headline bench at 100 and 13 clients.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_native_resnet_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_native.log 2>&1 || { tail -30 gpurun_out/pt_native.log; exit 1; }
tail -1 gpurun_out/pt_native.log
for c in 100 13 100 13; do
  timeout -k 10 300 python -u bench.py --clients $c --steps 3 --warmup 1 > gpurun_out/bench_nc$c.log 2>&1 || { tail -20 gpurun_out/bench_nc$c.log; exit 1; }
  echo "C=$c $(grep -o '"value": [0-9.]*' gpurun_out/bench_nc$c.log)"
done
