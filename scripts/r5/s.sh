#!/bin/bash
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5s
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu_steps.sh \
 "FEDML_AMD_SIDE_WGRAD=0 FEDML_AMD_C3W_BATCH=0 timeout -k 10 300 python -u scripts/layer_prof.py --C 100 --dtype fp32 > gpurun_out/r5s/lp100.txt 2>&1" \
 "FEDML_AMD_SIDE_WGRAD=0 FEDML_AMD_C3W_BATCH=0 timeout -k 10 300 python -u scripts/layer_prof.py --C 13 --dtype fp32 > gpurun_out/r5s/lp13.txt 2>&1" \
 "timeout -k 10 400 python -u bench.py --clients 13 --steps 20 --warmup 5 > gpurun_out/r5s/bench13_long.txt 2>&1"
