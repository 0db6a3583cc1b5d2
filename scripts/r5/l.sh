#!/bin/bash
# round 5, call L: which change broke 2 ranks == 1 rank (deterministic, resnet_shallow, ragged)?
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5l
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
T="python -u -m pytest -v --timeout 600 --timeout-method thread -p no:cacheprovider"
bash scripts/gpu_steps.sh \
 "FEDML_AMD_C3W_BATCH=0 timeout -k 10 400 $T tests/test_rccl_dist_gpu.py -k two_ranks > gpurun_out/r5l/t_nobatch.txt 2>&1" \
 "timeout -k 10 400 $T tests/test_rccl_dist_gpu.py -k two_ranks > gpurun_out/r5l/t_default.txt 2>&1" \
 "timeout -k 10 600 $T tests/test_rccl_dist_gpu.py -k 'four or eight' > gpurun_out/r5l/t_48.txt 2>&1"
