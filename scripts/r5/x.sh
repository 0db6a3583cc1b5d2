#!/bin/bash
# round 5, call X: reproduce the deterministic multi-rank flake (whole test_rccl_dist_gpu.py, twice)
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5x
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
T="python -u -m pytest -v --timeout 600 --timeout-method thread -p no:cacheprovider tests/test_rccl_dist_gpu.py"
bash scripts/gpu_steps.sh \
 "timeout -k 10 400 $T > gpurun_out/r5x/run1.txt 2>&1" \
 "timeout -k 10 400 $T > gpurun_out/r5x/run2.txt 2>&1" \
 "FEDML_AMD_HIP_GRAPHS=0 timeout -k 10 400 $T > gpurun_out/r5x/run3_nographs.txt 2>&1"
