#!/bin/bash
# round 5, call M: deterministic multi-rank flake — batched wgrad on vs off, three runs each of the 8-rank rehearsal
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5m
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
T="python -u -m pytest -q --timeout 600 --timeout-method thread -p no:cacheprovider tests/test_rccl_dist_gpu.py -k eight"
bash scripts/gpu_steps.sh \
 "FEDML_AMD_C3W_BATCH=0 timeout -k 10 200 $T > gpurun_out/r5m/nob1.txt 2>&1" \
 "FEDML_AMD_C3W_BATCH=0 timeout -k 10 200 $T > gpurun_out/r5m/nob2.txt 2>&1" \
 "FEDML_AMD_C3W_BATCH=0 timeout -k 10 200 $T > gpurun_out/r5m/nob3.txt 2>&1" \
 "timeout -k 10 200 $T > gpurun_out/r5m/b1.txt 2>&1" \
 "timeout -k 10 200 $T > gpurun_out/r5m/b2.txt 2>&1" \
 "timeout -k 10 200 $T > gpurun_out/r5m/b3.txt 2>&1"
