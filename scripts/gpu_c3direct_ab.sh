#!/bin/bash
# A/B: 3x3 weight gradient straight into the OIHW arena (atomics) vs GEMM scratch + scatter pass.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_native_resnet_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_native.log 2>&1 || { tail -30 gpurun_out/pt_native.log; exit 1; }
tail -1 gpurun_out/pt_native.log
for d in 1 0 1 0; do
  for c in 100 13; do
    FEDML_AMD_C3_DIRECT_WGRAD=$d timeout -k 10 300 python -u bench.py --clients $c --steps 3 --warmup 1 > gpurun_out/bench_c3d$d_c$c.log 2>&1 || { tail -20 gpurun_out/bench_c3d$d_c$c.log; exit 1; }
    echo "direct=$d C=$c $(grep -o '"value": [0-9.]*' gpurun_out/bench_c3d$d_c$c.log)"
  done
done
