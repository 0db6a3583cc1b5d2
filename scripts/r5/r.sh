#!/bin/bash
# round 5, call R: per-step budgets (layer_prof, per-layer kernels: no side stream / batched wgrad) + driver-style bench
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5r
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu_steps.sh \
 "FEDML_AMD_SIDE_WGRAD=0 FEDML_AMD_C3W_BATCH=0 timeout -k 10 300 python -u scripts/layer_prof.py --C 100 > gpurun_out/r5r/lp100.txt 2>&1" \
 "FEDML_AMD_SIDE_WGRAD=0 FEDML_AMD_C3W_BATCH=0 timeout -k 10 300 python -u scripts/layer_prof.py --C 13 > gpurun_out/r5r/lp13.txt 2>&1" \
 "timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5r/bench_driver_style.txt 2>&1"
